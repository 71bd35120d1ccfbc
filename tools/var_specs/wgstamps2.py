# per-group stamps in gemm_wg<Conv2Wgrad>: entry, setup done, first stash done, first barrier
# passed, loop end (thread 0 of each 4-wave group of workgroup z=0/25, x=0)
G = "gemm.h"
COND = "(op.C == 512 && (blockIdx.z == 0 || blockIdx.z == 25) && blockIdx.x == 0 && (threadIdx.x & 255) == 0)"
def S(i):
    return f"if {COND} st[{i}] = __builtin_amdgcn_s_memtime(); "
VARIANTS = {
    "wgst2": [
        (G, "  __shared__ __attribute__((aligned(16))) T smem[STAGE * 2 * G];\n  const int grp = threadIdx.x >> 8,",
            "  __shared__ __attribute__((aligned(16))) T smem[STAGE * 2 * G];\n  long long st[8] = {0}; long long rt0 = __builtin_amdgcn_s_memrealtime(); " + S(0) + "\n  const int grp = threadIdx.x >> 8,"),
        (G, "  const int n_it = (m_end - m_beg + BM * G - 1) / (BM * G);\n",
            "  const int n_it = (m_end - m_beg + BM * G - 1) / (BM * G);\n  " + S(1) + "\n"),
        (G, "      stash(d, Xs);\n      __syncthreads();\n",
            "      stash(d, Xs);\n      if (it == 0) { " + S(2) + "}\n      __syncthreads();\n      if (it == 0) { " + S(3) + "}\n"),
        (G, "  if (grp != 0) return;\n  const float sc = op.out_scale;",
            "  " + S(4) + "\n  if " + COND + ' { printf("WGST2 z%d g%d rt0 %lld : %lld %lld %lld %lld\\n", (int)blockIdx.z, grp, rt0 % 100000000, st[1]-st[0], st[2]-st[0], st[3]-st[0], st[4]-st[0]); }\n  if (grp != 0) return;\n  const float sc = op.out_scale;'),
    ],
}
