# What the fp32 gradient slabs cost the step: knock out the reduction's slab
# loads, the producers' slab stores (gemm_wg: conv3 / conv2 / FC weight gradients; the fused
# backward's conv1 weight gradient), or both.  Timing only: the gradients are wrong.
import os, runpy
_r = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "redko.py"))
K, LD = _r["K"], _r["LD"]
G = "gemm.h"
C = "conv1.h"
GS = "        slab[((size_t)split * op.R + r + q) * op.C + c] = acc[i][j][q] * sc;"
CS = "        slab[so + (size_t)(16 * i + 4 * (lane >> 4) + q) * K1 + col] = acc[i][j][q] * (1.f / 255.f);"
NOLOAD = (K, LD, "    acc = f32x4{(float)r.v4, 0.f, 0.f, 0.f};")
NOSTORE = [(G, GS, "        if (acc[i][j][q] == 12345.f) slab[((size_t)split * op.R + r + q) * op.C + c] = acc[i][j][q] * sc;"),
           (C, CS, "        if (acc[i][j][q] == 12345.f) slab[so + (size_t)(16 * i + 4 * (lane >> 4) + q) * K1 + col] = acc[i][j][q] * (1.f / 255.f);")]
VARIANTS = {
    "slab_base": [],
    "slab_noload": [NOLOAD],
    "slab_nostore": NOSTORE,
    "slab_none": NOSTORE + [NOLOAD],
}
