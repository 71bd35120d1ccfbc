# knock-outs of the fp32 conv1 weight-gradient loop's LDS reads (timing only; results wrong),
# on top of the fp32 backward stamps (B32 lines)
import os, runpy
_b = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bwdstamps32c.py"))
ST = _b["VARIANTS"]["b32st"]
C = "conv1.h"
LA = "      for (int i = 0; i < 2; ++i) a[i] = lds_frag_k(dyt + kk * LDX + 16 * i, LDX, lane);\n    };\n    auto load_b"
LA_KO = "      for (int i = 0; i < 2; ++i) a[i] = V{(float)(kk + i), (float)lane, 1.f, 2.f};\n    };\n    auto load_b"
LB = "        for (int j = 0; j < 3; ++j) raw[4 * j + jj] = img[rr + 16 * j];"
LB_KO = "        for (int j = 0; j < 3; ++j) raw[4 * j + jj] = (uint32_t)(rr + 16 * j) & 255u;"
VARIANTS = {
    "wg_base": ST,
    "wg_ko_a": ST + [(C, LA, LA_KO)],
    "wg_ko_b": ST + [(C, LB, LB_KO)],
    "wg_ko_ab": ST + [(C, LA, LA_KO), (C, LB, LB_KO)],
}
