# s_memtime phase stamps of head_step_kernel (head.h), workgroup (0,0), thread 0 (wave 0): loads
# issued, h/z/Wh staged, heads MFMA, phase 2 (per-lane statistics, V-trace, dH row), phase 3 dz,
# phase 4 dWh + slab stores.  "HEAD" lines.
F = "head.h"
W = 'asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); '
C = "(blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)"
def S(i):
    return f'__builtin_amdgcn_sched_barrier(0); if {C} stamps[{i}] = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); '
VARIANTS = {
    "hstamps5": [
        (F, "  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n  const int T_ = a.T, S = a.S;",
            "  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n  long long stamps[16] = {0}; " + S(0) + "\n  const int T_ = a.T, S = a.S;"),
        (F, "  // ---- phase 1: stage h and z, zero dH, heads forward ----", S(1) + "\n  // ---- phase 1: stage h and z, zero dH, heads forward ----"),
        (F, "  for (int e = tid; e < 64 * LDD / VEC; e += 256) *reinterpret_cast<V*>(dHs + e * VEC) = F::zero();\n  __syncthreads();",
            "  for (int e = tid; e < 64 * LDD / VEC; e += 256) *reinterpret_cast<V*>(dHs + e * VEC) = F::zero();\n  __syncthreads();\n  " + S(2)),
        (F, "  if (a.heads_out && lead) {", S(3) + "\n  if (a.heads_out && lead) {"),
        (F, "    // dH[f][j] = ke p_j (log p_j + H) + kappa ([j == a] - p_j); dH[f][value] = dv", S(4) + "\n    // dH[f][j] = ke p_j (log p_j + H) + kappa ([j == a] - p_j); dH[f][value] = dv"),
        (F, "  // ---- phase 3: dz = gelu'(z)", S(5) + "\n  // ---- phase 3: dz = gelu'(z)"),
        (F, "  // ---- phase 4: dWh partial", W + S(6) + "\n  // ---- phase 4: dWh partial"),
        (F, "        a.slab_bh[(size_t)blockIdx.x * HEADS + tid] = bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid];\n    }\n    }\n  }\n}",
            "        a.slab_bh[(size_t)blockIdx.x * HEADS + tid] = bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid];\n    }\n    }\n  }\n  " + W + S(7) + '\n  if ' + C + ' { printf("HEAD"); for (int q = 1; q < 8; ++q) printf(" %lld", stamps[q] - stamps[0]); printf("\\n"); }\n}'),
    ],
}
