// Fused SAC chains: one workgroup per 16-transition row block runs a whole per-row dependency
// chain (Linear -> Linear -> head -> loss -> row-local backward GEMMs) with every hidden row
// tile in LDS, so the step is 12 launches instead of 24.
//
// Why per row block: in the SAC step every dependency between layers is row-local except the
// weight gradients (a sum over the batch) and the optimizer (global norm).  A 16-row tile of a
// 256x256 layer is 16x256x256 MACs -- a few hundred bf16 MFMA cycles per CU -- so the cost of
// a separate launch per layer (boundary + first-load latency, several us) dwarfs the layer.
// Inside one workgroup the layer's weight rows stream from L2 (every row block reads the same
// weights) and the activation operand comes from LDS.
//
// layer16: out[n][o] = epilogue(sum_k W[o][k] * in[n][k]) for the tile's 16 rows and all 256
// outputs; 4 waves, wave w owns o in [64w, 64w + 64) as four 16x16 MFMA tiles.  The operand
// roles, k order and epilogue arithmetic are those of gemm_jobs, so the fused and unfused
// steps produce bitwise-identical results (tests/test_gpu_sac.py).
#pragma once
#include "sac.h"

namespace sac {

template <typename T> struct Tile {
  static constexpr int PAD = 16 / (int)sizeof(T);
  static constexpr int LD = H + PAD;  // LDS row stride (elements): 528 B bf16 / 1040 B fp32,
                                      // 16-lane ds_read_b128 column reads are conflict-free
  static constexpr int SZ = 16 * LD;
};

// 16 rows (row0 .. row0 + 15, zero beyond nrows) of a [rows][ld] T matrix, K elements each
// (K a multiple of 16 bytes), into an LDS tile of stride Tile<T>::LD
template <typename T>
DEV void load_tile(const T* __restrict__ src, int ld, int K, int row0, int nrows, T* dst) {
  constexpr int VE = 16 / (int)sizeof(T);
  const int vpr = K / VE;
  for (int v = threadIdx.x; v < 16 * vpr; v += 256) {
    const int r = v / vpr, c = (v - r * vpr) * VE;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (row0 + r < nrows) x = *reinterpret_cast<const f32x4*>(src + (size_t)(row0 + r) * ld + c);
    *reinterpret_cast<f32x4*>(dst + r * Tile<T>::LD + c) = x;
  }
}

// MODE 0: relu(acc + bias);  MODE 1: acc masked by M[n][o] > 0 (ReLU backward).
// out (LDS tile, nullable), g_rm (row-major [N][256], nullable), g_t (transposed [.][ldt]).
template <typename T, int MODE>
DEV void layer16(const T* __restrict__ W, int ldw, int K, const float* __restrict__ bias,
                 const T* in, T* out, const T* M, int ldm, T* g_rm, T* g_t, int ldt, int row0,
                 int nrows) {
  using F = Frag<T>;
  typedef typename F::vec V;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int kl = F::KPL * g;
  const T* wp = W + (size_t)(64 * wave + c) * ldw + kl;
  const T* ip = in + c * Tile<T>::LD + kl;
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int CH = 4;
#pragma unroll 1
  for (int k0 = 0; k0 < K; k0 += CH * F::KSTEP) {
    V a[CH][4], b[CH];
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      const int k = k0 + s * F::KSTEP;
      if (k < K) {
        b[s] = *reinterpret_cast<const V*>(ip + k);
#pragma unroll
        for (int j = 0; j < 4; ++j) a[s][j] = F::load(wp + (size_t)16 * j * ldw + k);
      } else {
        b[s] = F::zero();
#pragma unroll
        for (int j = 0; j < 4; ++j) a[s][j] = F::zero();
      }
    }
#pragma unroll
    for (int s = 0; s < CH; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = F::mma(a[s][j], b[s], acc[j]);
  }
  const int n = row0 + c;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = 64 * wave + 16 * j + 4 * g;
    float v[4] = {acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i] + bias[o + i], 0.f);
    } else {
      float m[4];
      load4(M + (size_t)c * ldm + o, m);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = m[i] > 0.f ? v[i] : 0.f;
    }
    if (out) store4(out + c * Tile<T>::LD + o, v);
    if (n < nrows) {
      if (g_rm) store4(g_rm + (size_t)n * H + o, v);
      if (g_t) {
#pragma unroll
        for (int i = 0; i < 4; ++i) g_t[(size_t)(o + i) * ldt + n] = to_t<T>(v[i]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// chain_fwd_kernel: per row block and job, X -> Linear+ReLU -> Linear+ReLU -> head (policy
// sample / log-prob, or Q).  Critic phase: jobs {target actor on s1 -> a1 into xt, Q1 and Q2
// on [s|a] (hidden rows kept for the backward), actor on s -> pi into xp}; alpha phase:
// {actor on s}; inference: act / policy / Q.
// ---------------------------------------------------------------------------------------
struct ChainJob {
  const void* x;  // [N][ldx] (T) operand rows, K1 = padded fan-in (multiple of 32)
  int ldx, K1;
  const void* w1;  // [256][K1] (T)
  const float* b1;
  const void* w2;  // [256][256] (T)
  const float* b2;
  void *h1, *h1t, *h2, *h2t;  // optional global copies: row-major [N][256], transposed [.][ldt]
  HeadJob head;
};
struct ChainArgs {
  ChainJob j[4];
  int N, K, ldt;
};

template <typename T>
__global__ __launch_bounds__(256) void chain_fwd_kernel(const ChainArgs g) {
  __shared__ __attribute__((aligned(16))) T sX[Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH1[Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH2[Tile<T>::SZ];
  const ChainJob& J = g.j[blockIdx.y];
  const int row0 = blockIdx.x * 16;
  load_tile<T>((const T*)J.x, J.ldx, J.K1, row0, g.N, sX);
  __syncthreads();
  layer16<T, 0>((const T*)J.w1, J.K1, J.K1, J.b1, sX, sH1, nullptr, 0, (T*)J.h1, (T*)J.h1t, g.ldt,
                row0, g.N);
  __syncthreads();
  layer16<T, 0>((const T*)J.w2, H, H, J.b2, sH1, sH2, nullptr, 0, (T*)J.h2, (T*)J.h2t, g.ldt,
                row0, g.N);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int r = wave; r < 16; r += 4) {
    const int n = row0 + r;
    if (n < g.N) head_row<T>(J.head, sH2 + r * Tile<T>::LD, n, g.N, g.K, lane);
  }
}

// ---------------------------------------------------------------------------------------
// critic_chain_kernel (grid: row blocks x 2): both target-critic chains on [s1 | a1] -> t1, t2
// -> TD target, weights, losses, dQ (closs_row); then for Q network q = blockIdx.y:
// dh2 = dQ W3 (.) [h2 > 0] (LDS tile + transposed for dW2) and dh1 = (dh2 W2) (.) [h1 > 0]
// (transposed for dW1).  Both q blocks compute the same target (bitwise); q = 0 writes the
// metric terms and priorities.
// ---------------------------------------------------------------------------------------
struct CChainArgs {
  CLossArgs L;         // t-inputs unused (ht1/ht2); hc1/hc2 = critic hidden-2 rows (masks)
  const void* xt;      // [N][ldx] (T): [s1 | a1]
  int ldx, K1;
  const void *tw1[2], *tw2[2];  // target critic layers (T)
  const float *tb1[2], *tb2[2];
  const void* w2t[2];  // critic W2^T (T)
  const void* h1[2];   // critic hidden-1 rows [N][256] (T): dh1 masks
  void* dh1t[2];       // [256][ldt] (T)
};

template <typename T>
__global__ __launch_bounds__(256) void critic_chain_kernel(const CChainArgs g) {
  __shared__ __attribute__((aligned(16))) T sX[Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH1[Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH2[Tile<T>::SZ];
  __shared__ float st[2][16];
  const CLossArgs& a = g.L;
  const int q = blockIdx.y;
  const int row0 = blockIdx.x * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  load_tile<T>((const T*)g.xt, g.ldx, g.K1, row0, a.N, sX);
  __syncthreads();
#pragma unroll 1
  for (int c = 0; c < 2; ++c) {
    layer16<T, 0>((const T*)g.tw1[c], g.K1, g.K1, g.tb1[c], sX, sH1, nullptr, 0, nullptr, nullptr,
                  0, row0, a.N);
    __syncthreads();
    layer16<T, 0>((const T*)g.tw2[c], H, H, g.tb2[c], sH1, sH2, nullptr, 0, nullptr, nullptr, 0,
                  row0, a.N);
    __syncthreads();
    const float* w3 = c ? a.w3t2 : a.w3t1;
    const float* b3 = c ? a.b3t2 : a.b3t1;
    for (int r = wave; r < 16; r += 4) {
      float h[4];
      load4(sH2 + r * Tile<T>::LD + 4 * lane, h);
      const float t = dot_row(w3, lane, h) + b3[0];
      if (lane == 0) st[c][r] = t;
    }
    __syncthreads();
  }
  // TD target and dQ; dh2 of network q into the sH2 tile (rows beyond N stay zero)
  for (int r = wave; r < 16; r += 4) {
    const int n = row0 + r;
    float d[4] = {0.f, 0.f, 0.f, 0.f};
    if (n < a.N) {
      float dq[2];
      closs_row<T>(a, st[0][r], st[1][r], n, lane, q == 0, dq[0], dq[1]);
      dq_to_dh<T>(dq[q], q ? a.w3c2 : a.w3c1, (const T*)(q ? a.hc2 : a.hc1) + (size_t)n * H, lane, d);
      T* dt = (T*)(q ? a.dh2t : a.dh1t);
#pragma unroll
      for (int i = 0; i < 4; ++i) dt[(size_t)(4 * lane + i) * a.ldt + n] = to_t<T>(d[i]);
    }
    store4(sH2 + r * Tile<T>::LD + 4 * lane, d);
  }
  __syncthreads();
  layer16<T, 1>((const T*)g.w2t[q], H, H, nullptr, sH2, nullptr, (const T*)g.h1[q] + (size_t)row0 * H,
                H, nullptr, (T*)g.dh1t[q], a.ldt, row0, a.N);
}

// ---------------------------------------------------------------------------------------
// actor_chain_kernel: per row block, the actor step's row-local part.  Q1, Q2 chains on
// [s | pi] with the UPDATED critic -> actor loss term and dQ (aloss_row) -> dh2_q (in place in
// its LDS tile) -> dh1_q = (dh2_q W2_q) (.) [h1_q > 0] (in place) -> dpi and the policy-head
// backward (ahead_row) -> dha2 (LDS + transposed) -> dha1 = (dha2 W2a) (.) [ha1 > 0]
// (transposed for dW1a).
// ---------------------------------------------------------------------------------------
struct AChainArgs {
  ALossArgs L;       // hp1/hp2 unused (LDS); dh1/dh2 unused
  ABwdArgs B;        // dhp1/dhp2/dha2 unused (LDS); ha2 = actor hidden-2 rows (mask)
  const void* xp;    // [N][ldx] (T): [s | pi]
  int ldx, K1;
  const void *w1[2], *w2[2], *w2t[2];  // critic layers (T)
  const float *b1[2], *b2[2], *w3[2], *b3[2];
  const void* aw2t;  // actor W2^T (T)
  const void* ha1;   // actor hidden-1 rows [N][256] (T): dha1 mask
  void* dha1t;       // [256][ldt] (T)
};

template <typename T>
__global__ __launch_bounds__(256) void actor_chain_kernel(const AChainArgs g) {
  __shared__ __attribute__((aligned(16))) T sX[Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH1[2][Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH2[2][Tile<T>::SZ];
  __shared__ float sq[2][16];
  const ALossArgs& a = g.L;
  const int N = a.N;
  const int row0 = blockIdx.x * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  load_tile<T>((const T*)g.xp, g.ldx, g.K1, row0, N, sX);
  __syncthreads();
#pragma unroll 1
  for (int q = 0; q < 2; ++q) {
    layer16<T, 0>((const T*)g.w1[q], g.K1, g.K1, g.b1[q], sX, sH1[q], nullptr, 0, nullptr, nullptr,
                  0, row0, N);
    __syncthreads();
    layer16<T, 0>((const T*)g.w2[q], H, H, g.b2[q], sH1[q], sH2[q], nullptr, 0, nullptr, nullptr, 0,
                  row0, N);
    __syncthreads();
    for (int r = wave; r < 16; r += 4) {
      float h[4];
      load4(sH2[q] + r * Tile<T>::LD + 4 * lane, h);
      const float v = dot_row(g.w3[q], lane, h) + g.b3[q][0];
      if (lane == 0) sq[q][r] = v;
    }
  }
  __syncthreads();
  for (int r = wave; r < 16; r += 4) {
    const int n = row0 + r;
    float dq[2] = {0.f, 0.f};
    if (n < N) aloss_row(a, sq[0][r], sq[1][r], n, lane, dq[0], dq[1]);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      T* row = sH2[q] + r * Tile<T>::LD;
      float d[4];
      dq_to_dh<T>(dq[q], g.w3[q], row, lane, d);
      store4(row + 4 * lane, d);
    }
  }
  __syncthreads();
#pragma unroll 1
  for (int q = 0; q < 2; ++q)  // dh1_q in place of h1_q (each element read then written by one lane)
    layer16<T, 1>((const T*)g.w2t[q], H, H, nullptr, sH2[q], sH1[q], sH1[q], Tile<T>::LD, nullptr,
                  nullptr, 0, row0, N);
  __syncthreads();
  for (int r = wave; r < 16; r += 4) {
    const int n = row0 + r;
    T* dst = sH2[0] + r * Tile<T>::LD;  // dha2 tile (dh2 no longer needed)
    if (n < N) {
      ahead_row<T>(g.B, sH1[0] + r * Tile<T>::LD, sH1[1] + r * Tile<T>::LD,
                   (const T*)g.B.ha2 + (size_t)n * H, dst, n, lane);
    } else {
      float z[4] = {0.f, 0.f, 0.f, 0.f};
      store4(dst + 4 * lane, z);
    }
  }
  __syncthreads();
  layer16<T, 1>((const T*)g.aw2t, H, H, nullptr, sH2[0], nullptr, (const T*)g.ha1 + (size_t)row0 * H,
                H, nullptr, (T*)g.dha1t, a.ldt, row0, N);
}

}  // namespace sac
