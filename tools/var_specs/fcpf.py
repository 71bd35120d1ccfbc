# fp32 FC forward K loop (impala.hip FCF_PF / FCF_KACC): chunks in registers ahead of the one
# computed, accumulator chains per fragment.
H = "impala.hip"
OLD = "constexpr int FCF_PF = 2, FCF_KACC = 1;"
VARIANTS = {
    "fcpf1k1": [(H, OLD, "constexpr int FCF_PF = 1, FCF_KACC = 1;")],
    "fcpf2k2": [(H, OLD, "constexpr int FCF_PF = 2, FCF_KACC = 2;")],
    "fcpf1k2": [(H, OLD, "constexpr int FCF_PF = 1, FCF_KACC = 2;")],
}
