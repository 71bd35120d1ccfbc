# gemm_wg register-ring depth and phase knock-outs (timing only; knock-outs give wrong grads)
G = "gemm.h"
PDL = "class Op, int PD = 3>"
VARIANTS = {
    "pd1": [(G, PDL, "class Op, int PD = 1>")],
    "pd2": [(G, PDL, "class Op, int PD = 2>")],
    "pd3": [],
    "pd5": [(G, PDL, "class Op, int PD = 5>")],
    "nomma": [(G, "      if (active) {\n        if (do_bias)", "      if (active && m_end < 0) {\n        if (do_bias)")],
    "noload": [(G, "    const int m0 = m_beg + (it * G + grp) * BM;\n#pragma unroll\n    for (int i = 0; i < NX; ++i) {",
                   "    const int m0 = m_beg + (it * G + grp) * BM + (1 << 28);\n#pragma unroll\n    for (int i = 0; i < NX; ++i) {")],
    "noslab": [(G, "        slab[((size_t)split * op.R + r + q) * op.C + c] = acc[i][j][q] * sc;",
                   "        if (acc[i][j][q] == 12345.f) slab[((size_t)split * op.R + r + q) * op.C + c] = acc[i][j][q] * sc;")],
}
