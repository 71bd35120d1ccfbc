# phase stamps of conv12_fwd_s2d without measurement waits: s_memtime into LDS at phase points
# by wave 0 of each group (threads 0 and 256) of workgroup 0; printed at the end
F = "conv1.h"
def S(i):
    return (f'if (blockIdx.x == 0 && (threadIdx.x & 255) == 0) stl[(threadIdx.x >> 8) * 32 + ({i})] = '
            '__builtin_amdgcn_s_memtime(); ')
VARIANTS = {
    "fstamps3": [
        (F, "  const int kl = KPL * (lane >> 4);\n  uint4 nv[3];\n  if (f0 + grp < f1) c1_load_frame<T>(x + (size_t)(f0 + grp) * IMG, tid, nv);",
            "  const int kl = KPL * (lane >> 4);\n  __shared__ long long stl[64];\n  " + S(0) + "\n  uint4 nv[3];\n  if (f0 + grp < f1) c1_load_frame<T>(x + (size_t)(f0 + grp) * IMG, tid, nv);\n  "),
        (F, "    T* w1s = smem;", S(1) + "\n    T* w1s = smem;"),
        (F, "  // conv1 pixel tiles of this wave:", "  " + S(2) + "\n  // conv1 pixel tiles of this wave:"),
        (F, "    __syncthreads();  // the previous frame's readers of img / a1s are done\n    if (active) c1_stash_frame_rot<T, LDI>(img, tid, nv);\n    __syncthreads();",
            "    " + S("3 + 5 * it") + "\n    __syncthreads();  // the previous frame's readers of img / a1s are done\n    " + S("4 + 5 * it") + "\n    if (active) c1_stash_frame_rot<T, LDI>(img, tid, nv);\n    __syncthreads();\n    " + S("5 + 5 * it")),
        (F, "        (void)pg;\n      }\n    }\n    __syncthreads();",
            "        (void)pg;\n      }\n    }\n    " + S("6 + 5 * it") + "\n    __syncthreads();\n    " + S("7 + 5 * it")),
        (F, "          store4(act2 + ((size_t)f * P2 + pc) * OC2 + 16 * wave + 4 * (lane >> 4), v);\n        }\n      }\n    }\n  }\n}",
            "          store4(act2 + ((size_t)f * P2 + pc) * OC2 + 16 * wave + 4 * (lane >> 4), v);\n        }\n      }\n    }\n  }\n  " + S(30) + '\n  if (blockIdx.x == 0 && (threadIdx.x & 255) == 0) { printf("C12F%d", (int)(threadIdx.x >> 8)); for (int q = 1; q < 31; ++q) if (q < 19 || q == 30) printf(" %lld", stl[(threadIdx.x >> 8) * 32 + q] - stl[(threadIdx.x >> 8) * 32]); printf("\\n"); }\n}'),
    ],
}
