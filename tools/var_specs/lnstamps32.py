# s_memtime stamps of the pipelined fp32 LayerNorm / conv3-dgrad body (lnc3_body_f32r),
# workgroup 0, thread 0 (role 0, wave 0) and thread 256 (role 1, wave 4): start, LN / W3 issue
# done, the two prologue barriers, Z(f0), every step.  "LN" lines.
L = "lnc3.h"
C = "conv1.h"
def S(i, t=0):
    return (f"__builtin_amdgcn_sched_barrier(0); if (blockIdx.x == 0 && threadIdx.x == {t}) g_ln[{i}] = "
            "__builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); ")
VARIANTS = {
    "lnst": [
        (C, "namespace c1 {\nconstexpr int GRID", "__device__ long long g_ln[64];\nnamespace c1 {\nconstexpr int GRID"),
        (L, "  V wa[A ? 1 : 9][NKO];\n", "  " + S(0) + S(20, 256) + "\n  V wa[A ? 1 : 9][NKO];\n"),
        (L, "  __syncthreads();  // dact3 of every frame is in HBM / L2; the LN partials are in LDS\n",
            "  " + S(1) + S(21, 256) + "\n  __syncthreads();  // dact3 of every frame is in HBM / L2; the LN partials are in LDS\n  " + S(2) + "\n"),
        (L, "  __syncthreads();  // the combine area becomes the Z tiles\n",
            "  __syncthreads();  // the combine area becomes the Z tiles\n  " + S(3) + "\n"),
        (L, "    if (nF > 1) aload(f0 + 1);\n  }\n  __syncthreads();\n",
            "    if (nF > 1) aload(f0 + 1);\n  }\n  " + S(4) + S(22, 256) + "\n  __syncthreads();\n  " + S(5) + "\n"),
        (L, "      if (i + 2 < nF) aload(f0 + i + 2);\n    }\n    __syncthreads();\n  }\n",
            "      if (i + 2 < nF) aload(f0 + i + 2);\n    }\n    " + S("6 + 2 * i") + S("23 + i", 256) + "\n    __syncthreads();\n    " + S("7 + 2 * i") + "\n  }\n"),
        (L, "  lnc3_body<T>(dy, act3, stats, gam, w3, w3t, act2, dact3, dact2, ln_slab, N, fpw, (int)blockIdx.x, lds);\n    __syncthreads();",
            "  lnc3_body<T>(dy, act3, stats, gam, w3, w3t, act2, dact3, dact2, ln_slab, N, fpw, (int)blockIdx.x, lds);\n    __syncthreads();"),
        (C, "  if (is_a && nF > 0 && load_w2) c12_load_w2(w2t, wb, wave, lane);",
            "  " + S(30) + '\n  if (blockIdx.x == 0 && threadIdx.x == 0) { printf("LN"); for (int q = 1; q < 31; ++q) printf(" %lld", g_ln[q] ? g_ln[q] - g_ln[0] : -1); printf("\\n"); }\n  if (is_a && nF > 0 && load_w2) c12_load_w2(w2t, wb, wave, lane);'),
    ],
}
