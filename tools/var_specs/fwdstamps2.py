# phase stamps of conv12_fwd_s2d (workgroup 0, thread 0), cycles since kernel entry
F = "conv1.h"
W = 'asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); '
def S(i):
    return f'if (blockIdx.x == 0 && threadIdx.x == 0) stamps[{i}] = __builtin_amdgcn_s_memtime(); '
VARIANTS = {
    "fstamps2": [
        (F, "  const int kl = KPL * (lane >> 4);\n  uint4 nv[3];\n  if (f0 + grp < f1) c1_load_frame<T>(x + (size_t)(f0 + grp) * IMG, tid, nv);",
            "  const int kl = KPL * (lane >> 4);\n  long long stamps[24] = {0}; " + S(0) + "\n  uint4 nv[3];\n  if (f0 + grp < f1) c1_load_frame<T>(x + (size_t)(f0 + grp) * IMG, tid, nv);\n  "),
        (F, "    T* w1s = smem;", W + S(1) + "\n    T* w1s = smem;"),
        (F, "  // conv1 pixel tiles of this wave:", "  " + W + S(2) + "\n  // conv1 pixel tiles of this wave:"),
        (F, "    __syncthreads();  // the previous frame's readers of img / a1s are done\n    if (active) c1_stash_frame_rot<T, LDI>(img, tid, nv);\n    __syncthreads();",
            "    __syncthreads();  // the previous frame's readers of img / a1s are done\n    " + S("3 + 4 * it") + "\n    if (active) c1_stash_frame_rot<T, LDI>(img, tid, nv);\n    __syncthreads();\n    " + S("4 + 4 * it")),
        (F, "        (void)pg;\n      }\n    }\n    __syncthreads();",
            "        (void)pg;\n      }\n    }\n    " + S("5 + 4 * it") + "\n    __syncthreads();\n    " + S("6 + 4 * it")),
        (F, "          store4(act2 + ((size_t)f * P2 + pc) * OC2 + 16 * wave + 4 * (lane >> 4), v);\n        }\n      }\n    }\n  }\n}",
            "          store4(act2 + ((size_t)f * P2 + pc) * OC2 + 16 * wave + 4 * (lane >> 4), v);\n        }\n      }\n    }\n  }\n  " + S(20) + '\n  if (blockIdx.x == 0 && threadIdx.x == 0) { printf("C12F"); for (int q = 1; q < 21; ++q) printf(" %lld", stamps[q] ? stamps[q] - stamps[0] : -1); printf("\\n"); }\n}'),
    ],
}
