# fp32 FC forward tiles (impala.hip FCF_KW / FCF_BR x FCF_BC; gemm_tile_body KW = the 4 waves
# split each chunk's k-steps).  The product: KW, 32 x 48 (216 tiles at N = 1280).
H = "impala.hip"
OLD = "constexpr int FCF_BR = 16, FCF_BC = 80;"
VARIANTS = {
    "fckw_off": [(H, "constexpr bool FCF_KW = true;", "constexpr bool FCF_KW = false;")],
    "fckw_32": [(H, OLD, "constexpr int FCF_BR = 32, FCF_BC = 32;")],
    "fckw_64": [(H, OLD, "constexpr int FCF_BR = 32, FCF_BC = 64;")],
    "fckw_16x80": [(H, OLD, "constexpr int FCF_BR = 16, FCF_BC = 80;")],
    "fckw_16x96": [(H, OLD, "constexpr int FCF_BR = 16, FCF_BC = 96;")],
}
