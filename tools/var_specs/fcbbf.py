# bf16 fc_bwd_kernel at two workgroups per CU (ops.h FcBwdCfg, G = 2): weight-gradient tiles
# 64 x 128 (192 workgroups at the same 6 splits) beside 320 input-gradient tiles of 64 x 64 on
# 2 x 4 waves (78 KB): 512 workgroups.
O1 = "  static constexpr int DR = G == 2 ? 128 : FCB_DR32, DWR = G == 2 ? 4 : FCB_DWR32;"
O2 = "  static constexpr int DC = G == 2 ? 64 : FCB_DC32, DWC = G == 2 ? 2 : FCB_DWC32;"
O3 = "  static constexpr int WBC = G == 2 ? 256 : FCB_WBC32;"
VARIANTS = {
    "fcbbf_x2": [("ops.h", O1, "  static constexpr int DR = G == 2 ? 64 : FCB_DR32, DWR = G == 2 ? 2 : FCB_DWR32;"),
                 ("ops.h", O2, "  static constexpr int DC = G == 2 ? 64 : FCB_DC32, DWC = G == 2 ? 4 : FCB_DWC32;"),
                 ("ops.h", O3, "  static constexpr int WBC = G == 2 ? 128 : FCB_WBC32;")],
    "fcbbf_w128": [("ops.h", O3, "  static constexpr int WBC = G == 2 ? 128 : FCB_WBC32;")],
}
