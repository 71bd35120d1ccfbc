# fc_bwd_kernel's input-gradient tiles (FcDgrad, gemm_tile_body) with two K chunks held ahead.
F = "ops.h"
OLD = "    gemm_tile_body<T, C::DR, 64, C::DBK, C::DWR, 2, FcDgrad<T>>(od, n_rtiles, (int)blockIdx.x - nw,"
VARIANTS = {
    "fcdpf2": [(F, OLD, "    gemm_tile_body<T, C::DR, 64, C::DBK, C::DWR, 2, FcDgrad<T>, sizeof(T) == 4 ? 2 : 1>(od, n_rtiles, (int)blockIdx.x - nw,")],
}
