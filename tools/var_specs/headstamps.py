F = "head.h"
W = 'asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); '
C = "(blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)"
def S(i):
    return f'if {C} stamps[{i}] = __builtin_amdgcn_s_memtime(); '
VARIANTS = {
    "hstamps": [
        (F, "  // ---- every global load of the kernel is issued here",
            "  long long stamps[16] = {0}; " + S(0) + "\n  // ---- every global load of the kernel is issued here"),
        (F, "  // ---- phase 1: stage h and z, zero dH, heads forward ----", W + S(1) + "\n  // ---- phase 1: stage h and z, zero dH, heads forward ----"),
        (F, "  // ---- phase 2: loss head on wave 0 (one lane per (trajectory, t)) ----", S(2) + "\n  // ---- phase 2: loss head on wave 0 (one lane per (trajectory, t)) ----"),
        (F, "  __syncthreads();\n  // ---- phase 3:", "  __syncthreads();\n  " + S(3) + "\n  // ---- phase 3:"),
        (F, "  // ---- phase 4: dWh partial", W + S(4) + "\n  // ---- phase 4: dWh partial"),
        (F, "        a.slab_bh[(size_t)blockIdx.x * HEADS + tid] = bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid];\n    }\n    }\n  }\n}",
            "        a.slab_bh[(size_t)blockIdx.x * HEADS + tid] = bred[0][tid] + bred[1][tid] + bred[2][tid] + bred[3][tid];\n    }\n    }\n  }\n  " + W + S(5) + '\n  if ' + C + ' { printf("HEAD"); for (int q = 1; q < 6; ++q) printf(" %lld", stamps[q] - stamps[0]); printf("\\n"); }\n}'),
    ],
}
