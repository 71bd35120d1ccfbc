# s_memtime phase stamps of head_step_kernel (head.h, round-4 layout), workgroup (0,0), thread 0
# (wave 0): loads issued, h/z/Wh staged, heads MFMA, phase 2a (quad statistics), 2b (V-trace on
# wave 0), 2c (dH rows), phase 3 dz, phase 4 dWh + slab stores.  "HEAD6" lines.
F = "head.h"
W = 'asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); '
C = "(blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)"
def S(i):
    return f'__builtin_amdgcn_sched_barrier(0); if {C} stamps[{i}] = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); '
VARIANTS = {
    "hstamps6": [
        (F, "  const int T_ = a.T, S = a.S;\n  const int traj0",
            "  long long stamps[16] = {0}; " + S(0) + "\n  const int T_ = a.T, S = a.S;\n  const int traj0"),
        (F, "  // ---- phase 1: stage h and z, zero dH, heads forward ----", S(1) + "\n  // ---- phase 1: stage h and z, zero dH, heads forward ----"),
        (F, "  for (int e = tid; e < 64 * LDD / VEC; e += 256) *reinterpret_cast<V*>(dHs + e * VEC) = F::zero();\n  __syncthreads();",
            "  for (int e = tid; e < 64 * LDD / VEC; e += 256) *reinterpret_cast<V*>(dHs + e * VEC) = F::zero();\n  __syncthreads();\n  " + S(2)),
        (F, "  // ---- phase 2a:", S(3) + "\n  // ---- phase 2a:"),
        (F, "  // ---- phase 2b:", S(4) + "\n  // ---- phase 2b:"),
        (F, "  // ---- phase 2c:", S(5) + "\n  // ---- phase 2c:"),
        (F, "  // ---- phase 3: dz = gelu'(z)", S(6) + "\n  // ---- phase 3: dz = gelu'(z)"),
        (F, "  // ---- phase 4: dWh partial", W + S(7) + "\n  // ---- phase 4: dWh partial"),
        (F, "        a.slab_bh[(size_t)blockIdx.x * HEADS + tid] = bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid];\n    }\n    }\n  }\n}",
            "        a.slab_bh[(size_t)blockIdx.x * HEADS + tid] = bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid];\n    }\n    }\n  }\n  " + W + S(8) + '\n  if ' + C + ' { printf("HEAD6"); for (int q = 1; q < 9; ++q) printf(" %lld", stamps[q] - stamps[0]); printf("\\n"); }\n}'),
    ],
}
