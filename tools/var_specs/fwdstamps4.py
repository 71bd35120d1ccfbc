# phase stamps of conv12_fwd_s2d (restructured loop) without measurement waits: s_memtime into
# LDS by wave 0 of each group of workgroup 0; printed at the end (one line per group)
F = "conv1.h"
def S(i):
    return (f'if (blockIdx.x == 0 && (threadIdx.x & 255) == 0) stl[(threadIdx.x >> 8) * 32 + ({i})] = '
            '__builtin_amdgcn_s_memtime(); ')
VARIANTS = {
    "fstamps4": [
        (F, "  const int kl = KPL * (lane >> 4);\n  uint4 nv[3];\n  if (f0 + grp < f1) c1_load_frame<T>(x + (size_t)(f0 + grp) * IMG, tid, nv);",
            "  const int kl = KPL * (lane >> 4);\n  __shared__ long long stl[64];\n  " + S(0) + "\n  uint4 nv[3];\n  if (f0 + grp < f1) c1_load_frame<T>(x + (size_t)(f0 + grp) * IMG, tid, nv);\n  "),
        (F, "    T* w1s = smem;", S(1) + "\n    T* w1s = smem;"),
        (F, "  if (f0 + grp < f1) c1_stash_frame_rot<T, LDI>(img, tid, nv);\n  if (f0 + grp + G < f1)",
            "  " + S(2) + "\n  if (f0 + grp < f1) c1_stash_frame_rot<T, LDI>(img, tid, nv);\n  if (f0 + grp + G < f1)"),
        (F, "      c1_mma(accA, 0);\n", "      " + S("3 + 4 * it") + "\n      c1_mma(accA, 0);\n"),
        (F, "    __syncthreads();  // the act1 tile is complete; the image is free",
            "    " + S("4 + 4 * it") + "\n    __syncthreads();  // the act1 tile is complete; the image is free\n    " + S("5 + 4 * it")),
        (F, "    __syncthreads();  // the image holds the next frame; the act1 tile is free\n  }\n}",
            "    " + S("6 + 4 * it") + "\n    __syncthreads();  // the image holds the next frame; the act1 tile is free\n  }\n  " + S(30) + '\n  if (blockIdx.x == 0 && threadIdx.x == 0) { for (int g = 0; g < 2; ++g) { printf("C12F%d", g); for (int q = 1; q < 31; ++q) if (q < 15 || q == 30) printf(" %lld", stl[g * 32 + q] - stl[g * 32]); printf("\\n"); } }\n}'),
    ],
}
