# fp32 FC weight + input gradient launch (fc_bwd_kernel<float, 1>): its LDS is the larger of the
# weight-gradient body's (64 x 256 tile, 32-row chunks: 84 KB) and the dgrad tiles' (72 KB), so
# one workgroup fits per CU and the 576 work items run in ~2.25 rounds of 4 waves per CU.  With
# 16-row weight-gradient chunks (42 KB; the same k-step order, bitwise-equal slabs) two fit.
O = "ops.h"
VARIANTS = {
    "fcw_bm32": [],
    "fcw_bm16": [
        (O, "  static constexpr int SW = gemm_wg_smem<T, 64, 256, 32, G>();",
            "  static constexpr int WBM = sizeof(T) == 4 ? 16 : 32;  // weight-gradient chunk rows\n  static constexpr int SW = gemm_wg_smem<T, 64, 256, WBM, G>();"),
        (O, "    gemm_wg_body<T, 64, 256, 1, 4, 32, G, FcWgrad<T>>(ow, slab, slab_bias, mps, (int)blockIdx.x,",
            "    gemm_wg_body<T, 64, 256, 1, 4, C::WBM, G, FcWgrad<T>>(ow, slab, slab_bias, mps, (int)blockIdx.x,"),
    ],
}
