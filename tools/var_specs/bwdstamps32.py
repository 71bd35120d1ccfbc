# s_memtime phase stamps of the fused per-frame backward (block 0, wave 0), printed once per
# launch: lnc3 prologue, per frame LN / dact3 / Z / col2im, conv12 prologue, per frame stash /
# conv2 dgrad / conv1 wgrad.  Run with tools/run_stamps.sh (prints the "BWD" lines).
L = "lnc3.h"
C = "conv1.h"
def S(i):
    return f"if (blockIdx.x == 0 && threadIdx.x == 0) g_st[{i}] = __builtin_amdgcn_s_memtime(); "
VARIANTS = {
    "bwdst": [
        (C, "namespace c1 {\nconstexpr int GRID", "__device__ long long g_st[64];\nnamespace c1 {\nconstexpr int GRID"),
        (L, "  lnc3_body<T>(dy, act3, stats, gam, w3, act2, dact3, dact2, ln_slab, N, fpw, (int)blockIdx.x, lds);\n  __syncthreads();  // this workgroup's dact2",
            "  " + S(0) + "\n  lnc3_body<T>(dy, act3, stats, gam, w3, act2, dact3, dact2, ln_slab, N, fpw, (int)blockIdx.x, lds);\n  __syncthreads();  " + S(20) + "// this workgroup's dact2"),
        (L, "  const int n_it = (f1 - f0 + G - 1) / G;\n  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers of the cell grid / red are done",
            "  " + S(1) + "\n  const int n_it = (f1 - f0 + G - 1) / G;\n  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers of the cell grid / red are done\n    " + S("2 + 4 * it")),
        (L, "    if (lane == 0) { red[grp][wave][0] = s1; red[grp][wave][1] = s2; }\n    __syncthreads();",
            "    if (lane == 0) { red[grp][wave][0] = s1; red[grp][wave][1] = s2; }\n    __syncthreads();\n    " + S("3 + 4 * it")),
        (L, "      store4(d3s + p0 * LD3 + c0, o);\n    }\n    __syncthreads();",
            "      store4(d3s + p0 * LD3 + c0, o);\n    }\n    __syncthreads();\n    " + S("4 + 4 * it")),
        (L, "      }\n    }\n    __syncthreads();\n    if (active) {\n      // ---- col2im gather",
            "      }\n    }\n    __syncthreads();\n    " + S("5 + 4 * it") + "\n    if (active) {\n      // ---- col2im gather"),
        (C, "  const int n_it = (f1 - f0 + G - 1) / G;\n  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers are done",
            "  " + S(21) + "\n  const int n_it = (f1 - f0 + G - 1) / G;\n  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers are done\n    " + S("22 + 4 * it")),
        (C, "    if (tid < c1::NPIX) msk[tid] = nmk;\n    }\n    __syncthreads();",
            "    if (tid < c1::NPIX) msk[tid] = nmk;\n    }\n    __syncthreads();\n    " + S("23 + 4 * it")),
        (C, "    __syncthreads();  // (every group reaches it: no early exit for an idle group)",
            "    __syncthreads();  // (every group reaches it: no early exit for an idle group)\n    " + S("24 + 4 * it")),
        (C, "        for (int j = 0; j < 3; ++j) acc[i][j] = F::mma(fa[s2 & 1][i], fb[s2 & 1][j], acc[i][j]);\n    }\n  }",
            "        for (int j = 0; j < 3; ++j) acc[i][j] = F::mma(fa[s2 & 1][i], fb[s2 & 1][j], acc[i][j]);\n    }\n    " + S("25 + 4 * it") + "\n  }"),
        (C, "  __syncthreads();  // all groups are done with their tiles",
            "  __syncthreads();  // all groups are done with their tiles\n  " + S(50) + "\n  if (blockIdx.x == 0 && threadIdx.x == 0 && sizeof(T) == 4) { printf(\"BWD\"); for (int q = 1; q < 51; ++q) printf(\" %lld\", g_st[q] ? g_st[q] - g_st[0] : -1); printf(\"\\n\"); }"),
    ],
}
