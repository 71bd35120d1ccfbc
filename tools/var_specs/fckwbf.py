# bf16 FC forward with the fp32 tiling: 32 x 48 tiles (216 at N = 1280) whose 8 waves split
# the k-steps (KW; BK 256 = 8 k-steps of 32, one per wave per chunk)
H = "impala.hip"
VARIANTS = {
    "fckwbf_48": [(H, "    constexpr bool KW = sizeof(T) == 4 && FCF_KW;", "    constexpr bool KW = FCF_KW;")],
}
