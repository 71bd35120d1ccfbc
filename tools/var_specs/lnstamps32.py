# s_memtime stamps of the 8-wave fp32 LayerNorm / conv3-dgrad body (lnc3_body_f32), workgroup 0
# thread 0 (wave 0) and thread 256 (wave 4): prologue, per frame LN sums / dact3 / Z / gather.
# "LN" lines.
L = "lnc3.h"
C = "conv1.h"
def S(i, t=0):
    return (f"__builtin_amdgcn_sched_barrier(0); if (blockIdx.x == 0 && threadIdx.x == {t}) g_ln[{i}] = "
            "__builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); ")
VARIANTS = {
    "lnst": [
        (C, "namespace c1 {\nconstexpr int GRID", "__device__ long long g_ln[64];\nnamespace c1 {\nconstexpr int GRID"),
        (L, "  const bool ln = wave < 4;  // waves 0..3: the LayerNorm features\n", "  const bool ln = wave < 4;  // waves 0..3: the LayerNorm features\n  " + S(0) + "\n"),
        (L, "  for (int e = t; e < lc3::ZR / 4; e += 512)  // the Z tile's zero row\n", "  " + S(1) + S(2, 256) + "\n  for (int e = t; e < lc3::ZR / 4; e += 512)  // the Z tile's zero row\n"),
        (L, "    __syncthreads();  // the previous frame's readers of Z / dact3 / red are done\n",
            "    __syncthreads();  // the previous frame's readers of Z / dact3 / red are done\n    " + S("3 + 5 * (f - f0)") + "\n"),
        (L, "    if (f + 1 < f1) fetch(f + 1);\n    if (ln) {\n      const float S1",
            "    " + S("4 + 5 * (f - f0)") + "\n    if (f + 1 < f1) fetch(f + 1);\n    if (ln) {\n      const float S1"),
        (L, "    // ---- Z[p][tap][ci] = sum_oc dact3[p][oc] W3[oc][tap][ci] ----\n",
            "    " + S("5 + 5 * (f - f0)") + "\n    // ---- Z[p][tap][ci] = sum_oc dact3[p][oc] W3[oc][tap][ci] ----\n"),
        (L, "    // ---- col2im gather in a fixed (kh, kw) order + conv2's ReLU mask -> dact2 ----\n#pragma unroll\n    for (int r = 0; r < NGI; ++r) {\n      const int e = t + 512 * r;",
            "    " + S("6 + 5 * (f - f0)") + "\n    // ---- col2im gather in a fixed (kh, kw) order + conv2's ReLU mask -> dact2 ----\n#pragma unroll\n    for (int r = 0; r < NGI; ++r) {\n      const int e = t + 512 * r;"),
        (L, "  // ---- gamma / beta partials -> slab [2][1024] ----\n",
            "  " + S(40) + "\n  // ---- gamma / beta partials -> slab [2][1024] ----\n"),
        (L, "  lnc3_body<T>(dy, act3, stats, gam, w3, w3t, act2, dact3, dact2, ln_slab, N, fpw, (int)blockIdx.x, lds);\n  __syncthreads();",
            "  lnc3_body<T>(dy, act3, stats, gam, w3, w3t, act2, dact3, dact2, ln_slab, N, fpw, (int)blockIdx.x, lds);\n  __syncthreads();\n  " + S(41)
            + '\n  if (blockIdx.x == 0 && threadIdx.x == 0) { printf("LN"); for (int q = 1; q < 42; ++q) if (q < 30 || q >= 40) printf(" %lld", g_ln[q] ? g_ln[q] - g_ln[0] : -1); printf("\\n"); }'),
    ],
}
