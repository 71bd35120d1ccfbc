# fp32 gemm_tile k-contiguous row pad (gemm.h F32_ROW_PAD): 8 floats (product) vs the round-3 4.
F = "gemm.h"
OLD = "constexpr int F32_ROW_PAD = 8;"
VARIANTS = {"rowpad4": [(F, OLD, "constexpr int F32_ROW_PAD = 4;")]}
