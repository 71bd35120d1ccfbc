# s_memtime stamps inside the fp32 forward's per-frame stash phase (conv1.h conv12_fwd_body,
# G = 1), workgroup 0, thread 0: conv2 loop end, after the next image's LDS stash, after the
# frame-after-next's load issue, after the 4x4x1 act2 block, after the act2 tile stores, after
# the frame barrier.  "STASH it t0 t1 t2 t3 t4 t5" lines, clocks from the conv2 loop end.
F = "conv1.h"
def S(i):
    return (f"__builtin_amdgcn_sched_barrier(0); if (blockIdx.x == 0 && threadIdx.x == 0) sts[{i}] = "
            "__builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); ")
VARIANTS = {
    "fstash": [
        (F, "  const int kl = KPL * (lane >> 4);\n  uint4 nv[3];",
            "  const int kl = KPL * (lane >> 4);\n  long long sts[8] = {0};\n  uint4 nv[3];"),
        (F, "      if (f + G < f1) c1_stash_frame_rot<__bf16, ILDI>(img, tid, nv);\n      if (f + 2 * G < f1) c1_load_frame<T>(x + (size_t)(f + 2 * G) * IMG, tid, nv);\n      if constexpr (!W2REG) {\n        // the 4x4x1 blocks",
            "      " + S(0) + "\n      if (f + G < f1) c1_stash_frame_rot<__bf16, ILDI>(img, tid, nv);\n      " + S(1) + "\n      if (f + 2 * G < f1) c1_load_frame<T>(x + (size_t)(f + 2 * G) * IMG, tid, nv);\n      " + S(2) + "\n      if constexpr (!W2REG) {\n        // the 4x4x1 blocks"),
        (F, "          a2s[((f - f0) * A2F + cy * A2W + cx) * LDA2 + oc] = (T)v;\n        }\n      }\n",
            "          a2s[((f - f0) * A2F + cy * A2W + cx) * LDA2 + oc] = (T)v;\n        }\n      }\n      " + S(3) + "\n"),
        (F, "    __syncthreads();  // the image holds the next frame; the act1 tile is free\n  }",
            "    " + S(4) + "\n    __syncthreads();  // the image holds the next frame; the act1 tile is free\n    " + S(5)
            + '\n    if (blockIdx.x == 0 && threadIdx.x == 0 && sizeof(T) == 4) { printf("STASH %d", it); for (int q = 1; q < 6; ++q) printf(" %lld", sts[q] - sts[0]); printf("\\n"); }\n  }'),
    ],
}
