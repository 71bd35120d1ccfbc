F = "lnc3.h"
W = 'asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); '
def S(i):
    return f'if (blockIdx.x == 0 && threadIdx.x == 0) stamps[{i}] = __builtin_amdgcn_s_memtime(); '
VARIANTS = {
    "lstamps": [
        (F, "  // ---- per-frame inputs, prefetched one frame ahead ----",
            "  long long stamps[24] = {0}; " + S(0) + "\n  // ---- per-frame inputs, prefetched one frame ahead ----"),
        (F, "  // zero the cell grids once (the border stays zero)", W + S(1) + "\n  // zero the cell grids once (the border stays zero)"),
        (F, "    __syncthreads();  // the previous frame's readers of the cell grid / red are done",
            "    __syncthreads();  // the previous frame's readers of the cell grid / red are done\n    " + S("2 + 4 * it")),
        (F, "    if (f + G < f1) fetch(f + G);", "    " + S("3 + 4 * it") + "\n    if (f + G < f1) fetch(f + G);"),
        (F, "      // ---- conv3 dgrad from the LDS cell grid -> dact2 (conv2's ReLU mask) ----",
            "      " + S("4 + 4 * it") + "\n      // ---- conv3 dgrad from the LDS cell grid -> dact2 (conv2's ReLU mask) ----"),
        (F, "  // ---- gamma / beta partials: fixed-order combine of the groups -> slab [2][1024] ----",
            "  " + S(20) + "\n  // ---- gamma / beta partials: fixed-order combine of the groups -> slab [2][1024] ----"),
        (F, "  for (int e = (int)threadIdx.x; e < 2 * FLAT / 4; e += 256 * G)\n    *reinterpret_cast<f32x4*>(slab",
            "  " + S(21) + '\n  if (blockIdx.x == 0 && threadIdx.x == 0) { printf("LNC3"); for (int q = 1; q < 22; ++q) printf(" %lld", stamps[q] ? stamps[q] - stamps[0] : -1); printf("\\n"); }\n  for (int e = (int)threadIdx.x; e < 2 * FLAT / 4; e += 256 * G)\n    *reinterpret_cast<f32x4*>(slab'),
    ],
}
