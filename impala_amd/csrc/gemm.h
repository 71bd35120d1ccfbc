// Two MFMA GEMM skeletons cover every contraction of the learner step.
//
//  gemm_rc  : D[r][c] = sum_k A[r][k] * B(c, k)      (forward convs, FC, heads, all dgrads)
//             Both operands are k-contiguous, so every lane loads its fragment straight from
//             HBM/L2 with one 16-byte load (no LDS round trip); rows = output channels,
//             cols = pixels/frames, so each lane ends up with 4 consecutive channels of one
//             pixel -> one vector store into the channels-last activation.
//  gemm_wg  : D[r][c] = sum_m X(m, r) * Y(m, c)      (all weight gradients)
//             Reduction over pixels m; operands are m-strided in HBM, so a 32-deep m-chunk of
//             both is staged through LDS transposed ([r][m], [c][m]) and fragments are read
//             k-contiguous from LDS.  The m range is split over blockIdx.z; each split writes
//             an fp32 partial slab that reduce_grads() sums in a fixed order (deterministic).
#pragma once
#include "common.h"

template <typename T, int TR, int TC, class Op>
__global__ __launch_bounds__(256) void gemm_rc(const Op op) {
  using F = Frag<T>;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r0 = blockIdx.y * (16 * TR);
  const int cw = (blockIdx.x * 4 + wave) * (16 * TC);
  const int kl = F::KPL * (lane >> 4);
  typename Op::ColCtx cc[TC];
#pragma unroll
  for (int j = 0; j < TC; ++j) cc[j] = op.col_ctx(min(cw + 16 * j + (lane & 15), op.C - 1));
  const T* arow[TR];
#pragma unroll
  for (int i = 0; i < TR; ++i) arow[i] = op.a_row(r0 + 16 * i + (lane & 15), min(cw, op.C - 1));
  f32x4 acc[TR][TC];
#pragma unroll
  for (int i = 0; i < TR; ++i)
#pragma unroll
    for (int j = 0; j < TC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int k = 0; k < Op::K; k += F::KSTEP) {
    typename F::vec a[TR], b[TC];
#pragma unroll
    for (int i = 0; i < TR; ++i) a[i] = F::load(arow[i] + k + kl);
#pragma unroll
    for (int j = 0; j < TC; ++j) b[j] = op.load_b(cc[j], k + kl);
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
      for (int j = 0; j < TC; ++j) acc[i][j] = F::mma(a[i], b[j], acc[i][j]);
  }
#pragma unroll
  for (int j = 0; j < TC; ++j) {
    const int c = cw + 16 * j + (lane & 15);
    if (c >= op.C) continue;
#pragma unroll
    for (int i = 0; i < TR; ++i) {
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      op.store(r0 + 16 * i + 4 * (lane >> 4), c, v);
    }
  }
}

template <typename T, int BR, int BC, int WR, int WC, class Op>
__global__ __launch_bounds__(256) void gemm_wg(const Op op, float* __restrict__ slab,
                                               float* __restrict__ slab_bias, int m_per_split) {
  using F = Frag<T>;
  constexpr int BMK = 32;
  constexpr int LD = BMK + 16 / (int)sizeof(T);  // +16 B per row
  constexpr int TRW = BR / 16 / WR, TCW = BC / 16 / WC;
  static_assert(WR * WC == 4, "4 waves");
  static_assert(TRW >= 1 && TCW >= 1, "tile");
  __shared__ __attribute__((aligned(16))) T Xs[BR * LD];
  __shared__ __attribute__((aligned(16))) T Ys[BC * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c0 = blockIdx.x * BC, r0 = blockIdx.y * BR, split = blockIdx.z;
  const int m_beg = split * m_per_split;
  const int m_end = min(op.M, m_beg + m_per_split);
  const int wr = wave / WC, wc = wave % WC;
  const int kl = F::KPL * (lane >> 4);
  const bool do_bias = slab_bias != nullptr && blockIdx.x == 0;
  f32x4 acc[TRW][TCW];
#pragma unroll
  for (int i = 0; i < TRW; ++i)
#pragma unroll
    for (int j = 0; j < TCW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bias_acc = 0.f;
  for (int m0 = m_beg; m0 < m_end; m0 += BMK) {
    for (int e = tid; e < BR * BMK / 4; e += 256) {
      const int mm = e / (BR / 4), rr = (e % (BR / 4)) * 4;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (m0 + mm < m_end) op.load_x4(m0 + mm, r0 + rr, v);
#pragma unroll
      for (int i = 0; i < 4; ++i) Xs[(rr + i) * LD + mm] = (T)v[i];
    }
    for (int e = tid; e < BC * BMK / 4; e += 256) {
      const int mm = e / (BC / 4), cc = (e % (BC / 4)) * 4;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (m0 + mm < m_end && c0 + cc < op.C) op.load_y4(m0 + mm, c0 + cc, v);
#pragma unroll
      for (int i = 0; i < 4; ++i) Ys[(cc + i) * LD + mm] = (T)v[i];
    }
    __syncthreads();
    if (do_bias && tid < BR) {
#pragma unroll 8
      for (int mm = 0; mm < BMK; ++mm) bias_acc += (float)Xs[tid * LD + mm];
    }
#pragma unroll
    for (int kk = 0; kk < BMK; kk += F::KSTEP) {
      typename F::vec a[TRW], b[TCW];
#pragma unroll
      for (int i = 0; i < TRW; ++i)
        a[i] = F::load(&Xs[((wr * TRW + i) * 16 + (lane & 15)) * LD + kk + kl]);
#pragma unroll
      for (int j = 0; j < TCW; ++j)
        b[j] = F::load(&Ys[((wc * TCW + j) * 16 + (lane & 15)) * LD + kk + kl]);
#pragma unroll
      for (int i = 0; i < TRW; ++i)
#pragma unroll
        for (int j = 0; j < TCW; ++j) acc[i][j] = F::mma(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
  const float sc = op.out_scale;
#pragma unroll
  for (int j = 0; j < TCW; ++j) {
    const int c = c0 + (wc * TCW + j) * 16 + (lane & 15);
    if (c >= op.C) continue;
#pragma unroll
    for (int i = 0; i < TRW; ++i) {
      const int r = r0 + (wr * TRW + i) * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        slab[((size_t)split * op.R + r + q) * op.C + c] = acc[i][j][q] * sc;
    }
  }
  if (do_bias && tid < BR) slab_bias[(size_t)split * op.R + r0 + tid] = bias_acc;
}
