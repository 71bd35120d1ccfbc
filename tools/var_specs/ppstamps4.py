# s_memtime stamps of the two-group fp32 conv12 backward body after the k-split weight gradient
# (C12B32::WKS), workgroup 0: group A wave 0 (thread 0) per frame: top / before the barrier;
# group B wave 4 (thread 256) per step: top / weight gradient done (before its LDS staging
# stores).  One "PP" line: clocks from the body's start.
C = "conv1.h"
def S(i, t=0):
    return (f"__builtin_amdgcn_sched_barrier(0); if (blockIdx.x == 0 && threadIdx.x == {t}) g_pp[{i}] = "
            "__builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); ")
END = ("          slab[so + (size_t)(16 * i + 4 * (lane >> 4) + q) * K1 + col] = acc[0][i][j][q] * (1.f / 255.f);\n"
       "      }\n  }\n}\n")
VARIANTS = {
    "pp4": [
        (C, "namespace c1 {\nconstexpr int GRID", "__device__ long long g_pp[80];\nnamespace c1 {\nconstexpr int GRID"),
        (C, "  if (!is_a && nF > 0) stage(-1, 0, f0, 0);\n  __syncthreads();",
            "  if (!is_a && nF > 0) stage(-1, 0, f0, 0);\n  __syncthreads();\n  " + S(0)),
        (C, '      asm volatile("" : "+v"(sl), "+v"(zt8));', '      asm volatile("" : "+v"(sl), "+v"(zt8));\n      ' + S("1 + 2 * it")),
        (C, '        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");\n      }\n      __syncthreads();\n    }',
            '        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");\n      }\n      ' + S("2 + 2 * it") + '\n      __syncthreads();\n    }'),
        (C, "      StRegs sr;\n", "      " + S("40 + 2 * (it - 1)", 256) + "\n      StRegs sr;\n"),
        (C, "      stage_st(it < nF ? f0 + it : -1, it & 1,", "      " + S("41 + 2 * (it - 1)", 256) + "\n      stage_st(it < nF ? f0 + it : -1, it & 1,"),
        (C, END, END[:-2] + "  __syncthreads();\n  " + S(60)
            + '\n  if (blockIdx.x == 0 && threadIdx.x == 0) { printf("PP"); for (int q = 1; q < 61; ++q) if (q < 14 || (q >= 40 && q < 52) || q == 60) printf(" %lld", g_pp[q] ? g_pp[q] - g_pp[0] : -1); printf("\\n"); }\n}\n'),
    ],
}
