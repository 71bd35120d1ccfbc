# s_memtime stamps of the two-group fp32 conv12 backward body (conv12_bwd_body_f32), workgroup 0:
# group A wave 0 (thread 0) per frame: top / Z half 0 / gather half 0 / Z half 1 / gather half 1
# / staged; group B wave 4 (thread 256) per step: top / wgrad done.  "PP" lines.
C = "conv1.h"
LN = "lnc3.h"
def S(i, t=0):
    return (f"__builtin_amdgcn_sched_barrier(0); if (blockIdx.x == 0 && threadIdx.x == {t}) g_pp[{i}] = "
            "__builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); ")
VARIANTS = {
    "ppst": [
        (LN, "  const int ct = wave & 3;  // Z: ci tile\n", "  const int ct = wave & 3;  // Z: ci tile\n  " + S(61) + S(63, 256) + "\n"),
        (LN, "    for (int k = 0; k < 4; ++k)\n      if (f1 - f0 < k + 2) pre(k);\n", "    for (int k = 0; k < 4; ++k)\n      if (f1 - f0 < k + 2) pre(k);\n    " + S(62) + "\n"),
        (C, "namespace c1 {\nconstexpr int GRID", "__device__ long long g_pp[80];\nnamespace c1 {\nconstexpr int GRID"),
        (C, "  if (is_a && nF > 0 && load_w2) c12_load_w2(w2t, wb, wave, lane);", "  " + S(0) + "\n  if (is_a && nF > 0 && load_w2) c12_load_w2(w2t, wb, wave, lane);"),
        (C, "  if (!is_a && nF > 0) stage(-1, 0, f0, 0);\n  __syncthreads();",
            "  if (!is_a && nF > 0) stage(-1, 0, f0, 0);\n  __syncthreads();\n  " + S(1)),
        (C, '      asm volatile("" : "+v"(sl));', '      asm volatile("" : "+v"(sl));\n      ' + S("2 + 6 * it")),
        (C, "        // the previous half's gather reads of the Z tile are done before it is overwritten",
            "        " + S("3 + 6 * it + 2 * hf") + "\n        // the previous half's gather reads of the Z tile are done before it is overwritten"),
        (C, "        // half 1 reads back the partial sums this wave stored",
            "        " + S("4 + 6 * it + 2 * hf") + "\n        // half 1 reads back the partial sums this wave stored"),
        (C, "      stage(it < nF ? f0 + it : -1, it & 1, it + 1 < nF ? f0 + it + 1 : -1, (it + 1) & 1);\n",
            "      " + S("41 + 2 * (it - 1)", 256) + "\n      stage(it < nF ? f0 + it : -1, it & 1, it + 1 < nF ? f0 + it + 1 : -1, (it + 1) & 1);\n      " + S("52 + (it - 1)", 256) + "\n"),
        (C, '      const int b = (it - 1) & 1;\n      const float* dyt = dyt_buf(b);', '      ' + S("40 + 2 * (it - 1)", 256) + '\n      const int b = (it - 1) & 1;\n      const float* dyt = dyt_buf(b);'),
        (C, "          slab[so + (size_t)(16 * i + 4 * (lane >> 4) + q) * K1 + col] = acc[i][j][q] * (1.f / 255.f);\n      }\n  }\n}",
            "          slab[so + (size_t)(16 * i + 4 * (lane >> 4) + q) * K1 + col] = acc[i][j][q] * (1.f / 255.f);\n      }\n  }\n  __syncthreads();\n  " + S(60)
            + '\n  if (blockIdx.x == 0 && threadIdx.x == 0) { printf("PP"); for (int q = 1; q < 64; ++q) if (q < 32 || (q >= 40 && q < 58) || q >= 60) printf(" %lld", g_pp[q] ? g_pp[q] - g_pp[0] : -1); printf("\\n"); }\n}'),
    ],
}
