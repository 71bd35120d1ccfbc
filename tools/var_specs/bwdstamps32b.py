# s_memtime phase stamps of the fp32 fused backward (block 0, wave 0): lnc3 prologue and per
# frame LN / dact3 / Z, then conv12_bwd_body_f32: prologue, per frame stash / 4 classes /
# wgrad.  tools/run_stamps.sh prints the "BWD" lines.
L = "lnc3.h"
C = "conv1.h"
def S(i):
    return f"if (blockIdx.x == 0 && threadIdx.x == 0) g_st[{i}] = __builtin_amdgcn_s_memtime(); "
VARIANTS = {
    "bwdst": [
        (C, "namespace c1 {\nconstexpr int GRID", "__device__ long long g_st[96];\nnamespace c1 {\nconstexpr int GRID"),
        (L, "  lnc3_body<T>(dy, act3, stats, gam, w3, act2, dact3, dact2, ln_slab, N, fpw, (int)blockIdx.x, lds);\n  __syncthreads();  // this workgroup's dact2",
            "  " + S(0) + "\n  lnc3_body<T>(dy, act3, stats, gam, w3, act2, dact3, dact2, ln_slab, N, fpw, (int)blockIdx.x, lds);\n  __syncthreads();  " + S(20) + "// this workgroup's dact2"),
        (L, "  const int n_it = (f1 - f0 + G - 1) / G;\n  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers of the cell grid / red are done",
            "  " + S(1) + "\n  const int n_it = (f1 - f0 + G - 1) / G;\n  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers of the cell grid / red are done\n    " + S("2 + 3 * it")),
        (L, "      store4(d3s + p0 * LD3 + c0, o);\n    }\n    __syncthreads();",
            "      store4(d3s + p0 * LD3 + c0, o);\n    }\n    __syncthreads();\n    " + S("3 + 3 * it")),
        (L, "      }\n    }\n    __syncthreads();\n    if (active) {\n      // ---- col2im gather",
            "      }\n    }\n    __syncthreads();\n    " + S("4 + 3 * it") + "\n    if (active) {\n      // ---- col2im gather"),
        (C, "  const int cg = lane & 7, slot = lane >> 3;\n  for (int f = f0; f < f1; ++f) {\n    __syncthreads();  // the previous frame's readers are done",
            "  const int cg = lane & 7, slot = lane >> 3;\n  " + S(21) + "\n  for (int f = f0; f < f1; ++f) {\n    __syncthreads();  // the previous frame's readers are done\n    " + S("22 + 7 * (f - f0)")),
        (C, "    if (tid < c1::NPIX) msk[tid] = nmk;\n    __syncthreads();\n    if (f + 1 < f1) fetch(f + 1);",
            "    if (tid < c1::NPIX) msk[tid] = nmk;\n    __syncthreads();\n    " + S("23 + 7 * (f - f0)") + "\n    if (f + 1 < f1) fetch(f + 1);"),
        (C, "    asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");\n    // ---- col2im of class (py, px)",
            "    " + S("24 + 7 * (f - f0)") + "\n    asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");\n    " + S("25 + 7 * (f - f0)") + "\n    // ---- col2im of class (py, px)"),
        (C, "    __syncthreads();  // dY1 complete", "    __syncthreads();  // dY1 complete\n    " + S("26 + 7 * (f - f0)")),
        (C, "        for (int j = 0; j < 3; ++j) acc[i][j] = F::mma(fa[s2 & 1][i], fb[s2 & 1][j], acc[i][j]);\n    }\n  }\n  // conv1 bias: the 32 lanes",
            "        for (int j = 0; j < 3; ++j) acc[i][j] = F::mma(fa[s2 & 1][i], fb[s2 & 1][j], acc[i][j]);\n    }\n    " + S("27 + 7 * (f - f0)") + "\n  }\n  // conv1 bias: the 32 lanes"),
        (C, "  const size_t so = (size_t)wg * OC1 * K1;\n#pragma unroll\n  for (int i = 0; i < 2; ++i)\n#pragma unroll\n    for (int j = 0; j < 3; ++j) {\n      const int col = wave * c1::CH",
            "  " + S(60) + "\n  if (blockIdx.x == 0 && threadIdx.x == 0) { printf(\"BWD\"); for (int q = 1; q < 61; ++q) printf(\" %lld\", g_st[q] ? g_st[q] - g_st[0] : -1); printf(\"\\n\"); }\n  const size_t so = (size_t)wg * OC1 * K1;\n#pragma unroll\n  for (int i = 0; i < 2; ++i)\n#pragma unroll\n    for (int j = 0; j < 3; ++j) {\n      const int col = wave * c1::CH"),
    ],
}
