# s_memtime stamps of the fp32 LayerNorm / conv3-dgrad body (lnc3_body_f32r, round-4 layout),
# workgroup 0: thread 0 (role 0, wave 0) at every phase of every frame, thread 256 (role 1) at
# the end of its Z MFMAs.  "LN5 f t_top t_sums t_b2 t_ln t_b3 t_zdone(r1) t_b4 t_gather" lines,
# clocks from the body's start.
L = "lnc3.h"
C = "conv1.h"
def S(i, t=0):
    return (f"__builtin_amdgcn_sched_barrier(0); if (blockIdx.x == 0 && threadIdx.x == {t}) g_l5[{i}] = "
            "__builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); ")
VARIANTS = {
    "lnst5": [
        (C, "namespace c1 {\nconstexpr int GRID", "__device__ long long g_l5[128];\nnamespace c1 {\nconstexpr int GRID"),
        (L, "  if (f0 < f1) fetch(f0);\n  float gm[4]", "  " + S(0) + "\n  if (f0 < f1) fetch(f0);\n  float gm[4]"),
        (L, "    __syncthreads();  // the previous frame's readers of Z / dact3 / red are done\n",
            "    __syncthreads();  // the previous frame's readers of Z / dact3 / red are done\n    " + S("1 + 10 * (f - f0)") + "\n"),
        (L, "      if (lane == 0) { red[wave][0] = s1; red[wave][1] = s2; }\n    }\n    __syncthreads();\n",
            "      if (lane == 0) { red[wave][0] = s1; red[wave][1] = s2; }\n    }\n    " + S("2 + 10 * (f - f0)") + "\n    __syncthreads();\n    " + S("3 + 10 * (f - f0)") + "\n"),
        (L, "      store4(d3s + p0 * LD3 + c0, o);\n    }\n    __syncthreads();\n",
            "      store4(d3s + p0 * LD3 + c0, o);\n    }\n    " + S("4 + 10 * (f - f0)") + "\n    __syncthreads();\n    " + S("5 + 10 * (f - f0)") + "\n"),
        (L, "        *reinterpret_cast<f32x4*>(zs + (lane & 15) * lc3::ZR + tap * OC2 + 16 * ct + kl) = acc[tap];\n    }\n    __syncthreads();\n",
            "        *reinterpret_cast<f32x4*>(zs + (lane & 15) * lc3::ZR + tap * OC2 + 16 * ct + kl) = acc[tap];\n    }\n    " + S("6 + 10 * (f - f0)", 256) + "\n    __syncthreads();\n    " + S("7 + 10 * (f - f0)") + "\n"),
        (L, "        store4(dact2 + ((size_t)f * P2 + px) * OC2 + ci, o);\n      }\n    }\n  }\n",
            "        store4(dact2 + ((size_t)f * P2 + px) * OC2 + ci, o);\n      }\n    }\n    " + S("8 + 10 * (f - f0)") + "\n  }\n"),
        (C, "  if (is_a && nF > 0 && load_w2) c12_load_w2(w2t, wb, wave, lane);",
            '  if (blockIdx.x == 0 && threadIdx.x == 0) { for (int fr = 0; fr < 5; ++fr) { printf("LN5 %d", fr); for (int q = 1; q < 9; ++q) printf(" %lld", g_l5[10 * fr + q] ? g_l5[10 * fr + q] - g_l5[0] : -1); printf("\\n"); } }\n  if (is_a && nF > 0 && load_w2) c12_load_w2(w2t, wb, wave, lane);'),
    ],
}
