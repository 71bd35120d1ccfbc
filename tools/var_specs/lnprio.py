# Static wave priority in the pipelined fp32 LayerNorm / conv3-dgrad body: role 1 (LN + the
# scatter GEMM, the MFMA side) at s_setprio 1 for the whole body, so role 0's gather takes the
# issue slots its MFMAs leave (MI355X_MICROARCH.md "two waves per SIMD" items 2 and 4); or
# role 0 instead.
L = "lnc3.h"
A0 = "  V wa[LN ? 9 : 1][NKO];\n"
E0 = "  if constexpr (LN) {\n    // ---- gamma / beta partials -> slab [2][1024] ----\n"
VARIANTS = {
    "lnp_prio1": [(L, A0, "  if constexpr (LN) __builtin_amdgcn_s_setprio(1);\n" + A0),
                  (L, E0, "  if constexpr (LN) __builtin_amdgcn_s_setprio(0);\n" + E0)],
    "lnp_prio0": [(L, A0, "  if constexpr (!LN) __builtin_amdgcn_s_setprio(1);\n" + A0),
                  (L, E0, "  if constexpr (!LN) __builtin_amdgcn_s_setprio(0);\n" + E0)],
}
