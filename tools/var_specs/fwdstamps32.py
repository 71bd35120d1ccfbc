# s_memtime phase stamps of the fp32 fused forward (conv12_fwd_body, G = 1) in workgroup 0,
# wave 0: prologue, per frame conv1 / barrier / conv2 / stash+act2 stores, then the conv3 tail
# (W3 loads, MFMAs, LN epilogue).  Printed once per launch ("F32F" lines; tools/run_stamps.sh).
F = "conv1.h"
def S(i):
    return (f"__builtin_amdgcn_sched_barrier(0); if (blockIdx.x == 0 && threadIdx.x == 0) stl[{i}] = "
            "__builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); ")
VARIANTS = {
    "f32fst": [
        (F, "  const int kl = KPL * (lane >> 4);\n  uint4 nv[3];",
            "  const int kl = KPL * (lane >> 4);\n  __shared__ long long stl[64];\n  " + S(0) + "\n  uint4 nv[3];"),
        (F, "  const int n_it = (f1 - f0 + G - 1) / G;\n  // conv1 pixel tiles",
            "  " + S(1) + "\n  const int n_it = (f1 - f0 + G - 1) / G;\n  // conv1 pixel tiles"),
        (F, "      c1_mma(accA, 0);\n      c1_mma(accB, 2);\n      c1_epi(accA, 0, f);\n      c1_epi(accB, 2, f);\n",
            "      " + S("2 + 5 * it") + "\n      c1_mma(accA, 0);\n      " + S("40 + 4 * it") + "\n      c1_mma(accB, 2);\n      " + S("41 + 4 * it") + "\n      c1_epi(accA, 0, f);\n      " + S("42 + 4 * it") + "\n      c1_epi(accB, 2, f);\n"),
        (F, "    __syncthreads();  // the act1 tile is complete; the image is free",
            "    " + S("3 + 5 * it") + "\n    __syncthreads();  // the act1 tile is complete; the image is free\n    " + S("4 + 5 * it")),
        (F, "      if (f + G < f1) c1_stash_frame_rot<__bf16, ILDI>(img, tid, nv);",
            "      " + S("5 + 5 * it") + "\n      if (f + G < f1) c1_stash_frame_rot<__bf16, ILDI>(img, tid, nv);"),
        (F, "    __syncthreads();  // the image holds the next frame; the act1 tile is free\n  }",
            "    " + S("6 + 5 * it") + "\n    __syncthreads();  // the image holds the next frame; the act1 tile is free\n  }"),
        (F, "      const int nF = f1 - f0;\n      const LnLane lk", "      " + S(30) + "\n      const int nF = f1 - f0;\n      const LnLane lk"),
        (F, "      float* ets = reinterpret_cast<float*>(smem);\n#pragma unroll\n      for (int fr = 0; fr < FMAX; ++fr)\n        if (fr < nF)",
            "      " + S(31) + "\n      float* ets = reinterpret_cast<float*>(smem);\n#pragma unroll\n      for (int fr = 0; fr < FMAX; ++fr)\n        if (fr < nF)"),
        (F, "      // frames wave and wave + 4 (FMAX <= 8) in one interleaved pass\n",
            "      " + S(32) + "\n      // frames wave and wave + 4 (FMAX <= 8) in one interleaved pass\n"),
        (F, "        ln_frames_epilogue<T, 1>(ets + wave * P3 * LDE, 0, LDE, fr1, lane, lk, c3.act3, c3.y, c3.stats);\n      }\n",
            "        ln_frames_epilogue<T, 1>(ets + wave * P3 * LDE, 0, LDE, fr1, lane, lk, c3.act3, c3.y, c3.stats);\n      }\n      " + S(33)
            + '\n      if (blockIdx.x == 0 && threadIdx.x == 0) { printf("F32F"); for (int q = 1; q < 60; ++q) if (q < 27 || (q >= 30 && q < 34) || q >= 40) printf(" %lld", stl[q] - stl[0]); printf("\\n"); }\n'),
    ],
}
