# s_memtime stamps of the pipelined fp32 LayerNorm / conv3-dgrad body (lnc3_body_f32r),
# workgroup 0, lane 0 of wave 0 (role 0: gather) and wave 4 (role 1: LN + GEMM): per step
# it: [0] before the step's first barrier, [1] after it, [2] after the LN-sums barrier, [3] after
# the dact3 barrier.  Printed once ("LNP r<role> it <it>: ...", clocks from the body's entry).
L = "lnc3.h"
def S(i):
    return ("__builtin_amdgcn_sched_barrier(0); if (blockIdx.x == 0 && (threadIdx.x & 255) == 0) "
            f"g_lnp[(LN ? 64 : 0) + ({i})] = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); ")
VARIANTS = {
    "lnp_st": [
        (L, "namespace lc3 {", "__device__ long long g_lnp[128];\nnamespace lc3 {"),
        (L, "  const int kl = 4 * (lane >> 4);\n  const int j0 = 256 * wave + 4 * lane, p0 = j0 >> 6, c0 = j0 & 63;\n",
            "  const int kl = 4 * (lane >> 4);\n  const int j0 = 256 * wave + 4 * lane, p0 = j0 >> 6, c0 = j0 & 63;\n  " + S("63") + "\n"),
        (L, "    const int f = f0 + it;  // role 1: LN + GEMM of frame f (it < nF); role 0: gather of f - 1\n    __syncthreads();  // the previous step's readers of Z / dact3 / red are done\n",
            "    const int f = f0 + it;  // role 1: LN + GEMM of frame f (it < nF); role 0: gather of f - 1\n    " + S("4 * it") + "\n    __syncthreads();  // the previous step's readers of Z / dact3 / red are done\n    " + S("4 * it + 1") + "\n"),
        (L, "    __syncthreads();\n    // ---- role 1: dact3 -> HBM", "    __syncthreads();\n    " + S("4 * it + 2") + "\n    // ---- role 1: dact3 -> HBM"),
        (L, "    __syncthreads();\n    if constexpr (LN) {\n      // ---- Z[p]", "    __syncthreads();\n    " + S("4 * it + 3") + "\n    if constexpr (LN) {\n      // ---- Z[p]"),
        (L, "      __syncthreads();  // this workgroup's dact2 stores are visible to all its waves; LDS is reused\n      conv12_bwd_body_f32<0>",
            "      __syncthreads();  // this workgroup's dact2 stores are visible to all its waves; LDS is reused\n"
            "      if (blockIdx.x == 0 && threadIdx.x == 0) { for (int r = 0; r < 2; ++r) for (int i = 0; i < 7; ++i) printf(\"LNP r%d it %d: %lld %lld %lld %lld\\n\", r, i, g_lnp[64*r+4*i] - g_lnp[64*r+63], g_lnp[64*r+4*i+1] - g_lnp[64*r+63], g_lnp[64*r+4*i+2] - g_lnp[64*r+63], g_lnp[64*r+4*i+3] - g_lnp[64*r+63]); }\n"
            "      conv12_bwd_body_f32<0>"),
    ],
}
