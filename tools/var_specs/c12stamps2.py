F = "conv1.h"
W = 'asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); '
def S(i):
    return f'if (blockIdx.x == 0 && threadIdx.x == 0) stamps[{i}] = __builtin_amdgcn_s_memtime(); '
VARIANTS = {
    "stamps2": [
        (F, "  f32x4 acc[2][3];\n#pragma unroll\n  for (int i = 0; i < 2; ++i)\n#pragma unroll\n    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};\n  float bsum",
            "  long long stamps[24] = {0}; " + S(0) + "\n  f32x4 acc[2][3];\n#pragma unroll\n  for (int i = 0; i < 2; ++i)\n#pragma unroll\n    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};\n  float bsum"),
        (F, "  if (f0 + grp < f1) fetch(f0 + grp);  // the first frame is in flight during the prologue",
            "  if (f0 + grp < f1) fetch(f0 + grp);  // the first frame is in flight during the prologue\n  " + W + S(1)),
        (F, "    T* w2s = smem;\n    V wv[NPT];\n#pragma unroll\n    for (int i = 0; i < NPT; ++i) {\n      const int e = (int)threadIdx.x + i * NT;\n      wv[i] = *reinterpret_cast<const V*>(w2 + (size_t)e * VEC);\n    }",
            "    T* w2s = smem;\n    V wv[NPT];\n#pragma unroll\n    for (int i = 0; i < NPT; ++i) {\n      const int e = (int)threadIdx.x + i * NT;\n      wv[i] = *reinterpret_cast<const V*>(w2 + (size_t)e * VEC);\n    }\n    " + W + S(2)),
        (F, "  // zero the dY1 padding rows 225..255", S(3) + "\n  // zero the dY1 padding rows 225..255"),
        (F, "    __syncthreads();  // the previous frame's readers are done",
            "    __syncthreads();  // the previous frame's readers are done\n    " + W + S("4 + 4 * it")),
        (F, "    if (f + G < f1) fetch(f + G);", "    " + S("5 + 4 * it") + "\n    if (f + G < f1) fetch(f + G);"),
        (F, "    __syncthreads();  // (every group reaches it: no early exit for an idle group)",
            "    " + S("6 + 4 * it") + "\n    __syncthreads();  // (every group reaches it: no early exit for an idle group)\n    " + S("7 + 4 * it")),
        (F, "  // conv1 bias: sum each lane's partials", W + S(20) + "\n  // conv1 bias: sum each lane's partials"),
        (F, "  const size_t so = (size_t)blockIdx.x * OC1 * K1;",
            S(21) + '\n  if (blockIdx.x == 0 && threadIdx.x == 0) { printf("C12"); for (int q = 1; q < 22; ++q) printf(" %lld", stamps[q] ? stamps[q] - stamps[0] : -1); printf("\\n"); }\n  const size_t so = (size_t)blockIdx.x * OC1 * K1;'),
    ],
}
