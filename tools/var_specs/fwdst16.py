# s_memtime stamps of the bf16 forward (conv12_fwd_body), workgroup 0: thread 0 (group 0,
# wave 0) at kernel start, after the weight staging, after the first-frame barrier, around each
# iteration's two barriers, at the conv3 tail's W3 issue and after its barrier, at the end;
# thread 256 (group 1, wave 0) before each of its barriers.  One "FW" line per bf16 launch.
C = "conv1.h"
def S(i, t=0):
    return (f"__builtin_amdgcn_sched_barrier(0); if (blockIdx.x == 0 && threadIdx.x == {t}) g_fw[{i}] = "
            "__builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); ")
VARIANTS = {
    "fwdst16": [
        (C, "namespace c1 {\nconstexpr int GRID", "__device__ long long g_fw[64];\nnamespace c1 {\nconstexpr int GRID"),
        (C, "  const int n_it = (f1 - f0 + G - 1) / G;\n",
            "  " + S(1) + S(21, 256) + "\n  const int n_it = (f1 - f0 + G - 1) / G;\n"),
        (C, "  __syncthreads();\n  for (int it = 0; it < n_it; ++it) {\n",
            "  " + S(22, 256) + "\n  __syncthreads();\n  " + S(2) + "\n  for (int it = 0; it < n_it; ++it) {\n"),
        (C, "    __syncthreads();  // the act1 tile is complete; the image is free\n",
            "    " + S("3 + 4 * it") + S("40 + 2 * it", 256) + "\n    __syncthreads();  // the act1 tile is complete; the image is free\n    " + S("4 + 4 * it") + "\n"),
        (C, "    __syncthreads();  // the image holds the next frame; the act1 tile is free\n  }\n",
            "    " + S("5 + 4 * it") + S("41 + 2 * it", 256) + "\n    __syncthreads();  // the image holds the next frame; the act1 tile is free\n    " + S("6 + 4 * it") + "\n  }\n"),
        (C, "      const int gw = (int)threadIdx.x >> 6, nF = f1 - f0;\n      const LnLane lk = ln_lane_consts(lane, c3.b3, c3.gam, c3.bet);\n#pragma unroll\n      for (int i = 0; i < NPT3; ++i) {\n        const int e = (int)threadIdx.x + i * NT;\n        if (e < NV3) *reinterpret_cast<V*>(w3s",
            "      " + S(16) + "\n      const int gw = (int)threadIdx.x >> 6, nF = f1 - f0;\n      const LnLane lk = ln_lane_consts(lane, c3.b3, c3.gam, c3.bet);\n#pragma unroll\n      for (int i = 0; i < NPT3; ++i) {\n        const int e = (int)threadIdx.x + i * NT;\n        if (e < NV3) *reinterpret_cast<V*>(w3s"),
        (C, "      __syncthreads();\n      if (gw < nF) {\n        const int p = lane & 15, oy = p >> 2, ox = p & 3;\n        const T* a2f = a2s + (gw * A2F",
            "      __syncthreads();\n      " + S(17) + "\n      if (gw < nF) {\n        const int p = lane & 15, oy = p >> 2, ox = p & 3;\n        const T* a2f = a2s + (gw * A2F"),
        (C, "  conv12_fwd_body<T>(x, w1, b1, w2, b2, act1, mask, act2, N, fpw, c3, (int)blockIdx.x, smem);\n}\n",
            "  " + S(0) + "\n  conv12_fwd_body<T>(x, w1, b1, w2, b2, act1, mask, act2, N, fpw, c3, (int)blockIdx.x, smem);\n  "
            + S(18) + S(47, 256) + "\n  if constexpr (sizeof(T) == 2) {\n    __syncthreads();\n"
            '    if (blockIdx.x == 0 && threadIdx.x == 0) { printf("FW"); for (int q = 1; q < 19; ++q) printf(" %lld", g_fw[q] ? g_fw[q] - g_fw[0] : -1); printf(" |"); for (int q = 40; q < 48; ++q) printf(" %lld", g_fw[q] ? g_fw[q] - g_fw[0] : -1); printf("\\n"); }\n  }\n}\n'),
    ],
}
