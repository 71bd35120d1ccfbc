# s_memtime stamps (core clock) at the phase boundaries of the fused SAC chain kernels, block
# (0, 1) / (0, 0), thread 0; each stamp waits for that wave's own memory ops first.
F = "sac_fused.h"
W = 'asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); '


def S(i, c):
    return f'if ({c}) stamps[{i}] = __builtin_amdgcn_s_memtime(); '


def P(tag, n, c):
    return (f'if ({c}) {{ printf("{tag}"); for (int q = 1; q < {n}; ++q) '
            f'printf(" %lld", stamps[q] - stamps[0]); printf("\\n"); }}')


CF = "blockIdx.x == 0 && blockIdx.y == 1 && threadIdx.x == 0"
CC = "blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0"
CA = "blockIdx.x == 0 && threadIdx.x == 0"
VARIANTS = {
    "sacstamps": [
        # chain_fwd (job 1 = Q1)
        (F, "  const ChainJob& J = g.j[blockIdx.y];\n  const int row0 = blockIdx.x * 16;\n  constexpr int NB",
            "  long long stamps[8] = {0}; " + S(0, CF) + "\n  const ChainJob& J = g.j[blockIdx.y];\n  const int row0 = blockIdx.x * 16;\n  constexpr int NB"),
        (F, "  xt.store(sX);\n  __syncthreads();",
            "  xt.store(sX);\n  __syncthreads(); " + W + S(1, CF)),
        (F, "  __syncthreads();\n  epi16<T, 0>(mma_wf<T, NB>(w2, H, sH1), sBias[1], nom, sH2, (T*)J.h2, (T*)J.h2t, g.ldt, row0, g.N);\n  __syncthreads();",
            "  __syncthreads(); " + W + S(2, CF) + "\n  epi16<T, 0>(mma_wf<T, NB>(w2, H, sH1), sBias[1], nom, sH2, (T*)J.h2, (T*)J.h2t, g.ldt, row0, g.N);\n  __syncthreads(); " + W + S(3, CF)),
        (F, "                sH2 + r * Tile<T>::LD, row0 + r, g.N, g.K, lane, r);\n}",
            "                sH2 + r * Tile<T>::LD, row0 + r, g.N, g.K, lane, r);\n  " + W + S(4, CF) + P("FWD", 5, CF) + "\n}"),
        # critic chain
        (F, "  const CLossArgs& a = g.L;\n  const int q = blockIdx.y;",
            "  long long stamps[8] = {0}; " + S(0, CC) + "\n  const CLossArgs& a = g.L;\n  const int q = blockIdx.y;"),
        (F, "  xr.store(sX);\n  __syncthreads();\n  const float nom[4] = {0.f, 0.f, 0.f, 0.f};\n#pragma unroll\n  for (int c = 0;",
            "  xr.store(sX);\n  __syncthreads(); " + W + S(1, CC) + "\n  const float nom[4] = {0.f, 0.f, 0.f, 0.f};\n#pragma unroll\n  for (int c = 0;"),
        (F, "    if (lane == 0) st[c][r] = t;\n    __syncthreads();\n  }",
            "    if (lane == 0) st[c][r] = t;\n    __syncthreads(); " + W + S(2, CC) + "stamps[2+c] = stamps[2]; \n  }"),
        (F, "    store4(sH2 + r * Tile<T>::LD + 4 * lane, d);\n  }\n  __syncthreads();\n  epi16<T, 1>(mma_wf<T, NB>(w2, H, sH2), nullptr, h1m, nullptr, nullptr, (T*)g.dh1t[q], a.ldt, row0, a.N);\n}",
            "    store4(sH2 + r * Tile<T>::LD + 4 * lane, d);\n  }\n  __syncthreads(); " + W + S(4, CC) + "\n  epi16<T, 1>(mma_wf<T, NB>(w2, H, sH2), nullptr, h1m, nullptr, nullptr, (T*)g.dh1t[q], a.ldt, row0, a.N);\n  " + W + S(5, CC) + P("CRIT", 6, CC) + "\n}"),
        # actor chain
        (F, "  const ALossArgs& a = g.L;\n  ABwdArgs bb = g.B;",
            "  long long stamps[8] = {0}; " + S(0, CA) + "\n  const ALossArgs& a = g.L;\n  ABwdArgs bb = g.B;"),
        (F, "  bb.wm = sWh[0]; bb.wl = sWh[1];\n  __syncthreads();",
            "  bb.wm = sWh[0]; bb.wl = sWh[1];\n  __syncthreads(); " + W + S(1, CA)),
        (F, "    if (lane == 0) sq[q][r] = v;\n  }\n  __syncthreads();",
            "    if (lane == 0) sq[q][r] = v;\n  }\n  __syncthreads(); " + W + S(2, CA)),
        (F, "      store4(row + 4 * lane, d);\n    }\n  }\n  __syncthreads();",
            "      store4(row + 4 * lane, d);\n    }\n  }\n  __syncthreads(); " + W + S(3, CA)),
        (F, "    epi16<T, 1>(acc, nullptr, m, sH1[q], nullptr, nullptr, 0, row0, N);\n  }\n  __syncthreads();",
            "    epi16<T, 1>(acc, nullptr, m, sH1[q], nullptr, nullptr, 0, row0, N);\n  }\n  __syncthreads(); " + W + S(4, CA)),
        (F, "      store4(dst + 4 * lane, z);\n    }\n  }\n  __syncthreads();",
            "      store4(dst + 4 * lane, z);\n    }\n  }\n  __syncthreads(); " + W + S(5, CA)),
        (F, "  epi16<T, 1>(mma_wf<T, NB>(w2, H, sH2[0]), nullptr, ha1m, nullptr, nullptr, (T*)g.dha1t, a.ldt, row0, N);\n}",
            "  epi16<T, 1>(mma_wf<T, NB>(w2, H, sH2[0]), nullptr, ha1m, nullptr, nullptr, (T*)g.dha1t, a.ldt, row0, N);\n  " + W + S(6, CA) + P("ACT", 7, CA) + "\n}"),
    ],
}
