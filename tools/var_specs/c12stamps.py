F = "conv1.h"
W = 'asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); '
def S(i):
    return f'if (blockIdx.x == 0 && threadIdx.x == 0) stamps[{i}] = __builtin_amdgcn_s_memtime(); '
VARIANTS = {
    "stamps": [
        (F, "  f32x4 acc[2][3];\n#pragma unroll\n  for (int i = 0; i < 2; ++i)\n#pragma unroll\n    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};\n  float bsum",
            "  long long stamps[24] = {0}; " + S(0) + "\n  f32x4 acc[2][3];\n#pragma unroll\n  for (int i = 0; i < 2; ++i)\n#pragma unroll\n    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};\n  float bsum"),
        (F, "  // zero the dY1 padding rows 225..255", S(1) + "\n  // zero the dY1 padding rows 225..255"),
        (F, "    __syncthreads();  // the previous frame's readers are done",
            "    __syncthreads();  // the previous frame's readers are done\n    " + W + S("2 + 5 * it")),
        (F, "    if (f + G < f1) fetch(f + G);", "    " + S("3 + 5 * it") + "\n    if (f + G < f1) fetch(f + G);"),
        (F, "    __syncthreads();  // (every group reaches it: no early exit for an idle group)",
            "    __syncthreads();  // (every group reaches it: no early exit for an idle group)\n    " + S("4 + 5 * it")),
        (F, "  // conv1 bias: sum each lane's partials", W + S(20) + "\n  // conv1 bias: sum each lane's partials"),
        (F, "  const size_t so = (size_t)blockIdx.x * OC1 * K1;",
            S(21) + '\n  if (blockIdx.x == 0 && threadIdx.x == 0) printf("C12 n_it=%d w2=%lld | %lld %lld %lld | %lld %lld %lld | %lld %lld %lld | loopend=%lld comb=%lld\\n", n_it, stamps[1]-stamps[0], stamps[2]-stamps[0], stamps[3]-stamps[0], stamps[4]-stamps[0], stamps[7]-stamps[0], stamps[8]-stamps[0], stamps[9]-stamps[0], stamps[12]-stamps[0], stamps[13]-stamps[0], stamps[14]-stamps[0], stamps[20]-stamps[0], stamps[21]-stamps[0]);\n  const size_t so = (size_t)blockIdx.x * OC1 * K1;'),
    ],
}
