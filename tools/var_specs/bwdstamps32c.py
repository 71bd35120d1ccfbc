# s_memtime phase stamps of the fp32 fused per-frame backward (lnc3_conv12_bwd<float>) in
# workgroup 0, wave 0: lnc3 prologue, per frame LN sums / dact3 / Z / col2im; conv12 prologue,
# per frame stash / Z GEMM / gather / conv1 wgrad.  "B32" lines (tools/run_stamps.sh).
L = "lnc3.h"
C = "conv1.h"
def S(i):
    return (f"__builtin_amdgcn_sched_barrier(0); if (blockIdx.x == 0 && threadIdx.x == 0) g_st32[{i}] = "
            "__builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); ")
VARIANTS = {
    "b32st": [
        (L, "  // ---- gamma / beta partials: fixed-order combine of the groups -> slab [2][1024] ----",
            "  " + S(56) + "\n  // ---- gamma / beta partials: fixed-order combine of the groups -> slab [2][1024] ----"),
        (C, "  if (f0 < f1) fetch(f0);  // the first frame is in flight during the prologue",
            "  " + S(57) + "\n  if (f0 < f1) fetch(f0);  // the first frame is in flight during the prologue"),
        (C, "  // zero the dY1 rows no pixel writes (225..239), the dY2 pad rows (36..47) and each Z tile's",
            "  " + S(58) + "\n  // zero the dY1 rows no pixel writes (225..239), the dY2 pad rows (36..47) and each Z tile's"),
        (C, "namespace c1 {\nconstexpr int GRID", "__device__ long long g_st32[64];\nnamespace c1 {\nconstexpr int GRID"),
        (L, "  lnc3_body<T>(dy, act3, stats, gam, w3, w3t, act2, dact3, dact2, ln_slab, N, fpw, (int)blockIdx.x, lds);\n  __syncthreads();  // this workgroup's dact2",
            "  " + S(0) + "\n  lnc3_body<T>(dy, act3, stats, gam, w3, w3t, act2, dact3, dact2, ln_slab, N, fpw, (int)blockIdx.x, lds);\n  " + S(21) + "\n  __syncthreads();  // this workgroup's dact2"),
        (L, "  const int n_it = (f1 - f0 + G - 1) / G;\n  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers of the cell grid / red are done",
            "  " + S(1) + "\n  const int n_it = (f1 - f0 + G - 1) / G;\n  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers of the cell grid / red are done"),
        (L, "    if (lane == 0) { red[grp][wave][0] = s1; red[grp][wave][1] = s2; }\n    __syncthreads();",
            "    if (lane == 0) { red[grp][wave][0] = s1; red[grp][wave][1] = s2; }\n    __syncthreads();\n    " + S("2 + 4 * it")),
        (L, "      store4(d3s + p0 * LD3 + c0, o);\n    }\n    __syncthreads();",
            "      store4(d3s + p0 * LD3 + c0, o);\n    }\n    __syncthreads();\n    " + S("3 + 4 * it")),
        (L, "    __syncthreads();\n    if (active) {\n      // ---- col2im gather",
            "    __syncthreads();\n    " + S("4 + 4 * it") + "\n    if (active) {\n      // ---- col2im gather"),
        (L, "          store4(dact2 + ((size_t)f * P2 + px) * OC2 + ci, o);\n        }\n      }\n    }\n  }",
            "          store4(dact2 + ((size_t)f * P2 + px) * OC2 + ci, o);\n        }\n      }\n    }\n    " + S("5 + 4 * it") + "\n  }"),
        (C, "  const int tapoff = ((wave >> 1) * c1::GRID + (wave & 1)) * LDIB;  // conv1 wgrad: tap = wave",
            "  const int tapoff = ((wave >> 1) * c1::GRID + (wave & 1)) * LDIB;  // conv1 wgrad: tap = wave\n  " + S(22)),
        (C, "    if (tid < c1::NPIX) msk[tid] = nmk;\n    __syncthreads();\n    if (f + 1 < f1) fetch(f + 1);",
            "    " + S("23 + 5 * (f - f0)") + "\n    if (tid < c1::NPIX) msk[tid] = nmk;\n    __syncthreads();\n    " + S("24 + 5 * (f - f0)") + "\n    if (f + 1 < f1) fetch(f + 1);"),
        (C, '    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");\n    // ---- col2im of class',
            '    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");\n    ' + S("25 + 5 * (f - f0)") + '\n    // ---- col2im of class'),
        (C, "    __syncthreads();  // dY1 complete\n", "    " + S("26 + 5 * (f - f0)") + "\n    __syncthreads();  // dY1 complete\n    " + S("51 + (f - f0)") + "\n"),
        (C, "      __builtin_amdgcn_sched_barrier(0);\n    }\n  }\n  // conv1 bias",
            "      __builtin_amdgcn_sched_barrier(0);\n    }\n    " + S("27 + 5 * (f - f0)") + "\n  }\n  // conv1 bias"),
        (C, "        slab[so + (size_t)(16 * i + 4 * (lane >> 4) + q) * K1 + col] = acc[i][j][q] * (1.f / 255.f);\n    }\n}",
            "        slab[so + (size_t)(16 * i + 4 * (lane >> 4) + q) * K1 + col] = acc[i][j][q] * (1.f / 255.f);\n    }\n  " + S(50) + '\n  if (blockIdx.x == 0 && threadIdx.x == 0) { printf("B32"); for (int q = 1; q < 59; ++q) if (q < 48 || q >= 50) printf(" %lld", g_st32[q] ? g_st32[q] - g_st32[0] : -1); printf("\\n"); }\n}'),
    ],
}
