# fp32 FC input-gradient tiles inside fc_bwd_kernel (ops.h FCB_*32): the product runs 128 x 80
# tiles on 4 x 1 waves (128 tiles + the 128 weight-gradient workgroups = 256); fcbt_64 is the
# round-4 64 x 64 on 2 x 2 (320 tiles); fcbt_128x64 keeps 64-frame columns (160 tiles).
O = "constexpr int FCB_DR32 = 128, FCB_DC32 = 80, FCB_DWR32 = 4, FCB_DWC32 = 1;"
VARIANTS = {
    "fcbt_64": [("ops.h", O, "constexpr int FCB_DR32 = 64, FCB_DC32 = 64, FCB_DWR32 = 2, FCB_DWC32 = 2;")],
    "fcbt_128x64": [("ops.h", O, "constexpr int FCB_DR32 = 128, FCB_DC32 = 64, FCB_DWR32 = 2, FCB_DWC32 = 2;")],
}
