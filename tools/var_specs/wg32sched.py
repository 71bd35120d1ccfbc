# fp32 conv1 weight-gradient loop scheduling in conv12_bwd_body_f32: prefetch distance and
# sched_group_barrier interleaves (the compiler waits on each byte read right after issuing it)
C = "conv1.h"
LOOP = """    constexpr int NKK = L::NROW / KS;
    V fa[2][2], fb[2][3];
    frag(0, fa[0], fb[0]);
#pragma unroll
    for (int s2 = 0; s2 < NKK; ++s2) {
      if (s2 + 1 < NKK) frag((s2 + 1) * KS, fa[(s2 + 1) & 1], fb[(s2 + 1) & 1]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = F::mma(fa[s2 & 1][i], fb[s2 & 1][j], acc[i][j]);
    }"""
PD3 = """    constexpr int NKK = L::NROW / KS;
    V fa[3][2], fb[3][3];
    frag(0, fa[0], fb[0]);
    frag(KS, fa[1], fb[1]);
#pragma unroll
    for (int s2 = 0; s2 < NKK; ++s2) {
      if (s2 + 2 < NKK) frag((s2 + 2) * KS, fa[(s2 + 2) % 3], fb[(s2 + 2) % 3]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = F::mma(fa[s2 % 3][i], fb[s2 % 3][j], acc[i][j]);
    }"""
SG = """    constexpr int NKK = L::NROW / KS;
    V fa[2][2], fb[2][3];
    frag(0, fa[0], fb[0]);
#pragma unroll
    for (int s2 = 0; s2 < NKK; ++s2) {
      if (s2 + 1 < NKK) frag((s2 + 1) * KS, fa[(s2 + 1) & 1], fb[(s2 + 1) & 1]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = F::mma(fa[s2 & 1][i], fb[s2 & 1][j], acc[i][j]);
      if (s2 + 1 < NKK) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
#pragma unroll
        for (int u = 0; u < 12; ++u) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
    }"""
VARIANTS = {"base": [], "pd3": [(C, LOOP, PD3)], "sg": [(C, LOOP, SG)], "pd3sg": [(C, LOOP, PD3.replace("""        for (int j = 0; j < 3; ++j) acc[i][j] = F::mma(fa[s2 % 3][i], fb[s2 % 3][j], acc[i][j]);
    }""", """        for (int j = 0; j < 3; ++j) acc[i][j] = F::mma(fa[s2 % 3][i], fb[s2 % 3][j], acc[i][j]);
      if (s2 + 2 < NKK) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
#pragma unroll
        for (int u = 0; u < 12; ++u) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
    }"""))]}
