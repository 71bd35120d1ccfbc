# timing-only knock-outs of the weight-gradient GEMM loads (gemm_wg_body; wgrad23 + FC wgrad):
# Y (im2col) rows / X rows of every chunk read from the split's first chunk (L1/L2-resident)
# instead of streaming.  Results are wrong.
G = "gemm.h"
VARIANTS = {
    "wk_base": [],
    "wk_ysame": [(G, "      const int m = m0 + min(tid + i * 256, NYV - 1) / YV;\n",
                     "      const int m = m_beg + min(tid + i * 256, NYV - 1) / YV;\n")],
    "wk_both": [(G, "      const int m = m0 + min(tid + i * 256, NYV - 1) / YV;\n",
                    "      const int m = m_beg + min(tid + i * 256, NYV - 1) / YV;\n"),
                (G, "      const int m = m0 + (tid + i * 256) / (BR / VEC);\n",
                    "      const int m = m_beg + (tid + i * 256) / (BR / VEC);\n")],
}
