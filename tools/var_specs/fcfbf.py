# bf16 FC forward K loop (impala.hip): two 256-deep chunks in registers ahead (PF 2, as fp32)
H = "impala.hip"
VARIANTS = {
    "fcfbf_pf2": [(H, "    constexpr int PF = sizeof(T) == 4 ? FCF_PF : 1, KA = sizeof(T) == 4 ? FCF_KACC : 1;",
                   "    constexpr int PF = FCF_PF, KA = sizeof(T) == 4 ? FCF_KACC : 1;")],
}
