# fp32 conv weight-gradient (wgrad23) pipeline shape: chunk prefetch depth PD, chunk rows BM
O = "ops.h"
B3 = "gemm_wg_body<T, 64, 64, 2, 2, 32, G, Conv3Wgrad<T>>(o3"
B2 = "gemm_wg_body<T, 64, 128, 1, 4, 32, G, Conv2Wgrad<T>>(o2"
CF = "  static constexpr int S3 = gemm_wg_smem<T, 64, 64, 32, G>(), S2 = gemm_wg_smem<T, 64, 128, 32, G>();"


def v(pd, bm):
    bm = f"(sizeof(T) == 4 ? {bm} : 32)"
    pd = f"(sizeof(T) == 4 ? {pd} : 2)"
    return [(O, B3, f"gemm_wg_body<T, 64, 64, 2, 2, {bm}, G, Conv3Wgrad<T>, {pd}>(o3"),
            (O, B2, f"gemm_wg_body<T, 64, 128, 1, 4, {bm}, G, Conv2Wgrad<T>, {pd}>(o2"),
            (O, CF, f"  static constexpr int S3 = gemm_wg_smem<T, 64, 64, {bm}, G>(), S2 = gemm_wg_smem<T, 64, 128, {bm}, G>();")]


VARIANTS = {
    "base": [],
    "pd3": v(3, 32),
    "pd4": v(4, 32),
    "bm64": v(2, 64),
    "bm64pd3": v(3, 64),
    "bm16pd4": v(4, 16),
}
