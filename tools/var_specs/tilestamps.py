G = "gemm.h"
COND = "(Op::A_KMAJOR && Op::K == 576 && blockIdx.x == 0 && threadIdx.x == 0)"
def S(i):
    return f"if {COND} stamps[{i}] = __builtin_amdgcn_s_memtime(); "
VARIANTS = {
    "tstamps": [
        (G, "  const int kl = F::KPL * (lane >> 4);\n  set_ctx(ft);\n  fetch(0);",
            "  long long stamps[32] = {0}; " + S(0) + "\n  const int kl = F::KPL * (lane >> 4);\n  set_ctx(ft);\n  fetch(0);"),
        (G, "      stash(buf);\n      __syncthreads();\n",
            "      stash(buf);\n      __syncthreads();\n      if (t == ft) { " + S("1 + kc") + "}\n"),
        (G, "            op.store(cr0 + (wr * TRW + i) * 16 + 4 * (lane >> 4), c, v, ep[i][j]);\n          }\n        }\n      }\n    }\n  }\n}",
            "            op.store(cr0 + (wr * TRW + i) * 16 + 4 * (lane >> 4), c, v, ep[i][j]);\n          }\n        }\n      }\n    }\n  }\n  " + S(20) + "\n  if " + COND + ' { printf("TILE"); for (int q = 1; q < 21; ++q) printf(" %lld", stamps[q] ? stamps[q] - stamps[0] : -1); printf("\\n"); }\n}'),
    ],
}
