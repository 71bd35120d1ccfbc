# fp32 fc_bwd_kernel at two workgroups per CU (ops.h FCB_*32): FC weight-gradient tiles 64 x 128
# (256 workgroups at the same 8 splits, 51 KB) beside 256 input-gradient tiles of 64 x 80 on 4 x 1
# waves (78 KB): 512 workgroups of ~10k MFMA cycles, two per CU.
O = "constexpr int FCB_DR32 = 128, FCB_DC32 = 80, FCB_DWR32 = 4, FCB_DWC32 = 1;"
W = "constexpr int FCB_WBC32 = 256;"
VARIANTS = {
    "fcb2_x2": [("ops.h", O, "constexpr int FCB_DR32 = 64, FCB_DC32 = 80, FCB_DWR32 = 4, FCB_DWC32 = 1;"),
                ("ops.h", W, "constexpr int FCB_WBC32 = 128;")],
    "fcb2_w128": [("ops.h", W, "constexpr int FCB_WBC32 = 128;")],
}
