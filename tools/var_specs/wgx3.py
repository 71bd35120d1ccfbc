# A/B of the fp32 weight-gradient GEMM arithmetic (gemm.h gemm_wg_body): "wgf32" restores the
# v_mfma_f32_16x16x4_f32 path (fp32 LDS tiles); the product library runs the exact bf16x3 split.
F = "gemm.h"
VARIANTS = {
    "wgf32": [
        (F, "  if constexpr (sizeof(T) == 4) return 3 * (BM / 32) * x3_xplane<BR>() + BM * (BC + 4);",
            "  if constexpr (false) return 3 * (BM / 32) * x3_xplane<BR>() + BM * (BC + 4);"),
        (F, "  constexpr bool X3M = sizeof(T) == 4;  // fp32: exact bf16x3 split passes (mma_x3)",
            "  constexpr bool X3M = false;"),
    ],
}
