# s_memtime stamps inside gemm_wg<Conv2Wgrad> (op.C == 512) for workgroups 0, 100, 255,
# thread 0; plus s_memrealtime at entry / exit to see the launch skew across workgroups
G = "gemm.h"
COND = "(op.C == 512 && (blockIdx.z == 0 || blockIdx.z == 25 || blockIdx.z == 63) && blockIdx.x == 0 && threadIdx.x == 0)"
def S(i):
    return f"if {COND} st[{i}] = __builtin_amdgcn_s_memtime(); "
VARIANTS = {
    "wgst": [
        (G, "  __shared__ __attribute__((aligned(16))) T smem[STAGE * 2 * G];\n  const int grp = threadIdx.x >> 8,",
            "  __shared__ __attribute__((aligned(16))) T smem[STAGE * 2 * G];\n  long long st[40] = {0}; long long rt0 = __builtin_amdgcn_s_memrealtime(); " + S(0) + "\n  const int grp = threadIdx.x >> 8,"),
        (G, "  const int n_it = (m_end - m_beg + BM * G - 1) / (BM * G);\n",
            "  const int n_it = (m_end - m_beg + BM * G - 1) / (BM * G);\n  " + S(1) + "\n"),
        (G, "      stash(d, Xs);\n      __syncthreads();\n",
            "      stash(d, Xs);\n      " + S("3 + 2 * it") + "\n      __syncthreads();\n      " + S("4 + 2 * it") + "\n"),
        (G, "  if (grp != 0) return;\n  const float sc = op.out_scale;",
            "  " + S(30) + "\n  if (grp != 0) return;\n  const float sc = op.out_scale;"),
        (G, "        slab[((size_t)split * op.R + r + q) * op.C + c] = acc[i][j][q] * sc;\n    }\n  }\n}",
            "        slab[((size_t)split * op.R + r + q) * op.C + c] = acc[i][j][q] * sc;\n    }\n  }\n  " + S(31) + "\n  if " + COND + ' { long long rt1 = __builtin_amdgcn_s_memrealtime(); printf("WGST z%d rt0 %lld rt1 %lld n_it %d :", (int)blockIdx.z, rt0 % 100000000, rt1 % 100000000, n_it); for (int q = 1; q < 32; ++q) printf(" %lld", st[q] ? st[q] - st[0] : -1); printf("\\n"); }\n}'),
    ],
}
