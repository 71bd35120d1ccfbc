# knock-outs of the two-group body's conv1 weight-gradient loop (group B), with the PP stamps:
# no image byte reads / no dY1 fragment reads / no scheduling groups
import os, runpy
base = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ppstamps32.py"))["VARIANTS"]["ppst"]
C = "conv1.h"
U8 = ("          for (int jj = 0; jj < 4; ++jj) raw[4 * j + jj] = img[rr[jj] + 16 * j];",
      "          for (int jj = 0; jj < 4; ++jj) raw[4 * j + jj] = (uint32_t)(lane + jj + kk + 16 * j) & 255u;")
FA = ("        for (int i = 0; i < 2; ++i) a[i] = lds_frag_k(dyt + kk * LDX + 16 * i, LDX, lane);",
      "        for (int i = 0; i < 2; ++i) a[i] = V{(float)(lane + kk), (float)i, 1.f, 2.f};")
SG = ("        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU: the j = 0 conversions\n", "        if (false) {\n")
SG2 = ("          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read\n        }\n        __builtin_amdgcn_sched_barrier(0);\n      }\n      " ,
       "          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read\n        }\n        }\n        __builtin_amdgcn_sched_barrier(0);\n      }\n      ")
VARIANTS = {
    "pp_nou8": base + [(C,) + U8],
    "pp_nofa": base + [(C,) + FA],
    "pp_nosg": base + [(C,) + SG, (C,) + SG2],
}
