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
// Workgroups are 16 waves (1024 threads): in a layer wave w owns the 16x16 output tile
// o in [16w, 16w + 16); in a row phase wave w owns transition row w.  The small per-row
// operands (head weights, W3, the critic's action columns, noise, saved head values) are staged
// into LDS at kernel entry, so no row phase waits on a dependent global load.
//
// A layer: out[n][o] = epilogue(sum_k W[o][k] * in[n][k]) for the tile's 16 rows and all 256
// outputs (mma_wf + epi16).  The operand roles, k order and epilogue arithmetic are those of
// gemm_jobs, so the fused and unfused steps give bitwise-identical results (test_gpu_sac.py).
#pragma once
#include "sac.h"

namespace sac {

template <typename T> struct Tile {
  static constexpr int PAD = 16 / (int)sizeof(T);
  static constexpr int LD = H + PAD;  // LDS row stride (elements): 528 B bf16 / 1040 B fp32,
                                      // 16-lane ds_read_b128 column reads are conflict-free
  static constexpr int SZ = 16 * LD;
};

constexpr int FW = 16;  // waves per fused workgroup

// This wave's A fragments (weight rows [16w, 16w + 16)) for k-steps [0, NS * KSTEP) of a layer,
// loaded ahead of the layer that consumes them (one layer of look-ahead hides the L2/HBM
// latency of the next weights behind the current layer's epilogue and row phase).
template <typename T, int NS> struct WF {
  typename Frag<T>::vec a[NS];
};
template <typename T> struct WFN {  // 256-deep layers / first layers with K1 <= 64
  static constexpr int BIG = H / Frag<T>::KSTEP, SMALL = 64 / Frag<T>::KSTEP;
};
template <typename T, int NS>
DEV WF<T, NS> load_wf(const T* __restrict__ W, int ldw, int K) {
  using F = Frag<T>;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const T* wp = W + (size_t)(16 * wave + (lane & 15)) * ldw + F::KPL * (lane >> 4);
  WF<T, NS> w;
  // k-steps at or beyond K load the last real k-step again (mma_wf skips them): a per-element
  // "load or zero" select compiles to a branch and a vmcnt(0) wait per fragment
  if (K > 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s) w.a[s] = F::load(wp + min(s * F::KSTEP, K - F::KSTEP));
  } else {
#pragma unroll
    for (int s = 0; s < NS; ++s) w.a[s] = F::zero();
  }
  return w;
}
// acc = sum_k W[o][k] in[n][k] from prefetched fragments (same k order as gemm_jobs)
template <typename T, int NS>
DEV f32x4 mma_wf(const WF<T, NS>& w, int K, const T* in) {
  using F = Frag<T>;
  typedef typename F::vec V;
  const int lane = threadIdx.x & 63;
  const T* ip = in + (lane & 15) * Tile<T>::LD + F::KPL * (lane >> 4);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (s * F::KSTEP < K) acc = F::mma(w.a[s], *reinterpret_cast<const V*>(ip + s * F::KSTEP), acc);
  return acc;
}
// epilogue of a 16-row layer tile: MODE 0 relu(acc + bias) (bias in LDS), MODE 1 acc masked by
// m (the lane's 4 mask values) > 0; stores to the LDS tile / row-major / transposed copies
template <typename T, int MODE>
DEV void epi16(f32x4 acc, const float* bias, const float m[4], T* out, T* g_rm, T* g_t, int ldt,
               int row0, int nrows) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, o = 16 * wave + 4 * (lane >> 4), n = row0 + c;
  float v[4] = {acc[0], acc[1], acc[2], acc[3]};
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = MODE == 0 ? fmaxf(v[i] + bias[o + i], 0.f) : (m[i] > 0.f ? v[i] : 0.f);
  if (out) store4(out + c * Tile<T>::LD + o, v);
  if (n < nrows) {
    if (g_rm) store4(g_rm + (size_t)n * H + o, v);
    if (g_t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) g_t[(size_t)(o + i) * ldt + n] = to_t<T>(v[i]);
    }
  }
}
// the lane's 4 mask values of a layer tile from LDS (row c, features o..o+3)
template <typename T>
DEV void tile_mask(const T* tile, float m[4]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  load4(tile + (lane & 15) * Tile<T>::LD + 16 * wave + 4 * (lane >> 4), m);
}
// ... or from a global row-major [rows][256] matrix.  Rows beyond nrows read the last row (an
// unconditional load; see Reg): they only reach tile rows that are never stored.
template <typename T>
DEV void rows_mask(const T* rm, int row0, int nrows, float m[4]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = min(row0 + (lane & 15), nrows - 1);
  load4(rm + (size_t)n * H + 16 * wave + 4 * (lane >> 4), m);
}
// Prologue staging in two passes -- every global load of the prologue is issued first (into
// registers), then the LDS stores -- so the prologue costs one memory round trip, not one per
// staged array.  M = elements per thread (n <= M * 1024).  The loads are unconditional (index
// clamped to n - 1; store() writes only i < n): a per-element "load or 0" select makes hipcc
// branch around each load with a vmcnt(0) wait, which serialises the prologue.
template <int M> struct Reg {
  float v[M];
  DEV void load(const float* __restrict__ src, int n) {
    if (n <= 0) {  // wave-uniform
#pragma unroll
      for (int j = 0; j < M; ++j) v[j] = 0.f;
      return;
    }
#pragma unroll
    for (int j = 0; j < M; ++j) v[j] = src[min((int)threadIdx.x + j * FW * 64, n - 1)];
  }
  DEV void store(float* dst, int n) const {
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const int i = (int)threadIdx.x + j * FW * 64;
      if (i < n) dst[i] = v[j];
    }
  }
};
// one 16-byte vector per thread of a 16-row operand tile (16 x K elements, K*sizeof(T) <= 1 KB)
template <typename T> struct TileReg {
  f32x4 x;
  int r, c;
  bool ok;
  DEV void load(const T* __restrict__ src, int ld, int K, int row0, int nrows) {
    constexpr int VE = 16 / (int)sizeof(T);
    const int vpr = K / VE, v = (int)threadIdx.x;
    ok = v < 16 * vpr;
    r = ok ? v / vpr : 0;
    c = ok ? (v - r * vpr) * VE : 0;
    x = f32x4{0.f, 0.f, 0.f, 0.f};
    if (ok && row0 + r < nrows) x = *reinterpret_cast<const f32x4*>(src + (size_t)(row0 + r) * ld + c);
  }
  DEV void store(T* dst) const {
    if (ok) *reinterpret_cast<f32x4*>(dst + r * Tile<T>::LD + c) = x;
  }
};

// head operands staged into LDS (policy: fc_mean rows then fc_logstd rows, biases, the row
// block's noise; Q: W3 and b3), loaded in the prologue's single round trip
struct HeadStage {
  Reg<MAXK * H / (FW * 64)> wm, wl;
  Reg<1> b, b2, e;
  DEV void load(const HeadJob& J, int K, int row0, int N) {
    if (J.kind == HK_Q) {
      wm.load(J.wm, H);
      b.load(J.bm, 1);
      return;
    }
    wm.load(J.wm, K * H);
    wl.load(J.wl, K * H);
    b.load(J.bm, K);   // fc_mean bias (thread t < K) ...
    b2.load(J.bl, K);  // ... and fc_logstd bias, merged at store time
    const int rows = min(16, N - row0);
    e.load(J.eps ? J.eps + (size_t)row0 * K : nullptr, J.eps ? rows * K : 0);
  }
  // LDS copies: weights [2K][256] in sW (Q: W3 in row 0), biases in sB, noise rows in sE
  DEV void store(const HeadJob& J, int K, float* sW, float* sB, float* sE) const {
    if (J.kind == HK_Q) {
      wm.store(sW, H);
      b.store(sB, 1);
      return;
    }
    wm.store(sW, K * H);
    wl.store(sW + K * H, K * H);
    b.store(sB, K);
    b2.store(sB + K, K);
    e.store(sE, 16 * K);
  }
};

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
__global__ __launch_bounds__(1024) void chain_fwd_kernel(const ChainArgs g) {
  __shared__ __attribute__((aligned(16))) T sX[Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH1[Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH2[Tile<T>::SZ];
  __shared__ float sW[2 * MAXK * H], sB[2 * MAXK], sE[16 * MAXK], sBias[2][H];
  const ChainJob& J = g.j[blockIdx.y];
  const int row0 = blockIdx.x * 16;
  constexpr int NB = WFN<T>::BIG, NS = WFN<T>::SMALL;
  const bool small = J.K1 <= 64;
  // issue order = use order (vmcnt retires loads in order): staged operands, W1, then W2,
  // whose stream overlaps the LDS staging and the first layer
  HeadStage hs;
  hs.load(J.head, g.K, row0, g.N);
  Reg<1> b1, b2;
  b1.load(J.b1, H);
  b2.load(J.b2, H);
  TileReg<T> xt;
  xt.load((const T*)J.x, J.ldx, J.K1, row0, g.N);
  WF<T, NS> w1 = load_wf<T, NS>((const T*)J.w1, J.K1, small ? J.K1 : 0);
  WF<T, NB> w2 = load_wf<T, NB>((const T*)J.w2, H, H);
  hs.store(J.head, g.K, sW, sB, sE);
  b1.store(sBias[0], H);
  b2.store(sBias[1], H);
  xt.store(sX);
  __syncthreads();
  const float nom[4] = {0.f, 0.f, 0.f, 0.f};
  if (small) {
    epi16<T, 0>(mma_wf<T, NS>(w1, J.K1, sX), sBias[0], nom, sH1, (T*)J.h1, (T*)J.h1t, g.ldt, row0, g.N);
  } else {  // wide first layer (64 < K1 <= 256): its fragments are fetched here
    const WF<T, NB> wk = load_wf<T, NB>((const T*)J.w1, J.K1, J.K1);
    epi16<T, 0>(mma_wf<T, NB>(wk, J.K1, sX), sBias[0], nom, sH1, (T*)J.h1, (T*)J.h1t, g.ldt, row0, g.N);
  }
  __syncthreads();
  epi16<T, 0>(mma_wf<T, NB>(w2, H, sH1), sBias[1], nom, sH2, (T*)J.h2, (T*)J.h2t, g.ldt, row0, g.N);
  __syncthreads();
  const int lane = threadIdx.x & 63, r = threadIdx.x >> 6;
  if (row0 + r < g.N)
    head_row<T>(J.head, sW, sB, sW + g.K * H, sB + g.K, J.head.eps ? sE : nullptr,
                sH2 + r * Tile<T>::LD, row0 + r, g.N, g.K, lane, r);
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
__global__ __launch_bounds__(1024) void critic_chain_kernel(const CChainArgs g) {
  __shared__ __attribute__((aligned(16))) T sX[Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH1[Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH2[Tile<T>::SZ];
  __shared__ float st[2][16], sW3[4][H], sB3[2], sBias[4][H];
  constexpr int NB = WFN<T>::BIG, NS = WFN<T>::SMALL;
  const CLossArgs& a = g.L;
  const int q = blockIdx.y;
  const int row0 = blockIdx.x * 16;
  const int lane = threadIdx.x & 63, r = threadIdx.x >> 6, n = row0 + r;
  const bool small = g.K1 <= 64;
  // everything this block reads from memory is requested up front, in use order
  // (rows beyond N load row N - 1 -- no branch around the loads -- and are never used)
  const int nc = min(n, a.N - 1);
  const CRow crow = load_crow(a, nc);
  const float la = a.log_alpha[0];
  float h2m[4], h1m[4];
  load_row<T>(q ? a.hc2 : a.hc1, H, nc, lane, h2m);
  rows_mask<T>((const T*)g.h1[q], row0, a.N, h1m);
  Reg<1> w3[4], bs[4];
  w3[0].load(a.w3t1, H);
  w3[1].load(a.w3t2, H);
  w3[2].load(a.w3c1, H);
  w3[3].load(a.w3c2, H);
  bs[0].load(g.tb1[0], H);
  bs[1].load(g.tb2[0], H);
  bs[2].load(g.tb1[1], H);
  bs[3].load(g.tb2[1], H);
  const float b3a = a.b3t1[0], b3b = a.b3t2[0];
  TileReg<T> xr;
  xr.load((const T*)g.xt, g.ldx, g.K1, row0, a.N);
  WF<T, NS> w1 = load_wf<T, NS>((const T*)g.tw1[0], g.K1, small ? g.K1 : 0);
  WF<T, NB> w2 = load_wf<T, NB>((const T*)g.tw2[0], H, H);
  const float wm = a.wmax[0];  // IS-weight normaliser (pack_kernel; 1 without probabilities)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w3[i].store(sW3[i], H);
    bs[i].store(sBias[i], H);
  }
  if (threadIdx.x < 2) sB3[threadIdx.x] = threadIdx.x ? b3b : b3a;
  xr.store(sX);
  __syncthreads();
  const float nom[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    f32x4 acc = small ? mma_wf<T, NS>(w1, g.K1, sX)
                      : mma_wf<T, NB>(load_wf<T, NB>((const T*)g.tw1[c], g.K1, g.K1), g.K1, sX);
    if (c == 0) w1 = load_wf<T, NS>((const T*)g.tw1[1], g.K1, small ? g.K1 : 0);
    epi16<T, 0>(acc, sBias[2 * c], nom, sH1, nullptr, nullptr, 0, row0, a.N);
    __syncthreads();
    acc = mma_wf<T, NB>(w2, H, sH1);
    w2 = load_wf<T, NB>((const T*)(c == 0 ? g.tw2[1] : g.w2t[q]), H, H);  // next big layer
    epi16<T, 0>(acc, sBias[2 * c + 1], nom, sH2, nullptr, nullptr, 0, row0, a.N);
    __syncthreads();
    float h[4];
    load4(sH2 + r * Tile<T>::LD + 4 * lane, h);
    const float t = dot_row(sW3[c], lane, h) + sB3[c];
    if (lane == 0) st[c][r] = t;
    __syncthreads();
  }
  // TD target and dQ; dh2 of network q into the sH2 tile (rows beyond N zero)
  {
    float d[4] = {0.f, 0.f, 0.f, 0.f};
    if (n < a.N) {
      float dq[2];
      closs_row<T>(a, crow, expf(la), wm, st[0][r], st[1][r], n, lane, q == 0,
                   dq[0], dq[1]);
      dq_to_dh(dq[q], sW3[2 + q], h2m, lane, d);
      T* dt = (T*)(q ? a.dh2t : a.dh1t);
#pragma unroll
      for (int i = 0; i < 4; ++i) dt[(size_t)(4 * lane + i) * a.ldt + n] = to_t<T>(d[i]);
    }
    store4(sH2 + r * Tile<T>::LD + 4 * lane, d);
  }
  __syncthreads();
  epi16<T, 1>(mma_wf<T, NB>(w2, H, sH2), nullptr, h1m, nullptr, nullptr, (T*)g.dh1t[q], a.ldt, row0, a.N);
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
__global__ __launch_bounds__(1024) void actor_chain_kernel(const AChainArgs g) {
  __shared__ __attribute__((aligned(16))) T sX[Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH1[2][Tile<T>::SZ];
  __shared__ __attribute__((aligned(16))) T sH2[2][Tile<T>::SZ];
  __shared__ float sq[2][16], sW3[2][H], sB3[2], sBias[4][H];
  __shared__ float sA[2][MAXK * H];   // critic action columns, [k][o]
  __shared__ float sWh[2][MAXK * H];  // actor fc_mean / fc_logstd rows
  __shared__ float sS[4 * 16 * MAXK], sE[16 * MAXK], sG[16][2 * MAXK];
  constexpr int NB = WFN<T>::BIG, NS = WFN<T>::SMALL;
  const ALossArgs& a = g.L;
  ABwdArgs bb = g.B;  // operands redirected into LDS
  const int N = a.N, K = bb.K, DK = bb.D + bb.K;
  const int row0 = blockIdx.x * 16;
  const int lane = threadIdx.x & 63, r = threadIdx.x >> 6, n = row0 + r;
  const bool small = g.K1 <= 64;
  const float la = a.log_alpha[0];
  // (rows beyond N load row N - 1 -- no branch around the loads -- and are never used)
  const int nc = min(n, N - 1);
  const float logp = a.logp[nc];
  float hv[4], ha1m[4];
  load_row<T>(bb.ha2, H, nc, lane, hv);
  rows_mask<T>((const T*)g.ha1, row0, N, ha1m);
  constexpr int MK = MAXK * H / (FW * 64);
  Reg<1> w3[2], bs[4];
  w3[0].load(g.w3[0], H);
  w3[1].load(g.w3[1], H);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    bs[2 * q].load(g.b1[q], H);
    bs[2 * q + 1].load(g.b2[q], H);
  }
  const float b3a = g.b3[0][0], b3b = g.b3[1][0];
  float ca[2][MK];  // critic action columns, gathered [k][o] from [o][D + k] (index clamped:
                    // unconditional loads, only i < K * H is stored)
#pragma unroll
  for (int j = 0; j < MK; ++j) {
    const int i = min((int)threadIdx.x + j * FW * 64, K * H - 1), k = i / H, o = i - k * H;
    ca[0][j] = bb.w1c1[(size_t)o * DK + bb.D + k];
    ca[1][j] = bb.w1c2[(size_t)o * DK + bb.D + k];
  }
  Reg<MK> whm, whl;
  whm.load(bb.wm, K * H);
  whl.load(bb.wl, K * H);
  const size_t NK = (size_t)N * K;
  const int rows = min(16, N - row0);
  Reg<1> sv[4], ev;
#pragma unroll
  for (int j = 0; j < 4; ++j) sv[j].load(bb.save + j * NK + (size_t)row0 * K, rows * K);
  ev.load(bb.eps + (size_t)row0 * K, rows * K);
  TileReg<T> xr;
  xr.load((const T*)g.xp, g.ldx, g.K1, row0, N);
  WF<T, NS> w1 = load_wf<T, NS>((const T*)g.w1[0], g.K1, small ? g.K1 : 0);
  WF<T, NB> w2 = load_wf<T, NB>((const T*)g.w2[0], H, H);
  // ---- LDS stores (one round trip after the loads above were issued)
  w3[0].store(sW3[0], H);
  w3[1].store(sW3[1], H);
#pragma unroll
  for (int i = 0; i < 4; ++i) bs[i].store(sBias[i], H);
  if (threadIdx.x < 2) sB3[threadIdx.x] = threadIdx.x ? b3b : b3a;
#pragma unroll
  for (int j = 0; j < MK; ++j) {
    const int i = (int)threadIdx.x + j * FW * 64;
    if (i < K * H) {
      sA[0][i] = ca[0][j];
      sA[1][i] = ca[1][j];
    }
  }
  whm.store(sWh[0], K * H);
  whl.store(sWh[1], K * H);
#pragma unroll
  for (int j = 0; j < 4; ++j) sv[j].store(sS + j * 16 * K, 16 * K);
  ev.store(sE, 16 * K);
  xr.store(sX);
  bb.w1c1 = sA[0]; bb.w1c2 = sA[1];
  bb.w1_so = 1; bb.w1_sk = H; bb.w1_off = 0;
  bb.wm = sWh[0]; bb.wl = sWh[1];
  __syncthreads();
  const float nom[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    f32x4 acc = small ? mma_wf<T, NS>(w1, g.K1, sX)
                      : mma_wf<T, NB>(load_wf<T, NB>((const T*)g.w1[q], g.K1, g.K1), g.K1, sX);
    if (q == 0) w1 = load_wf<T, NS>((const T*)g.w1[1], g.K1, small ? g.K1 : 0);
    epi16<T, 0>(acc, sBias[2 * q], nom, sH1[q], nullptr, nullptr, 0, row0, N);
    __syncthreads();
    acc = mma_wf<T, NB>(w2, H, sH1[q]);
    w2 = load_wf<T, NB>((const T*)(q == 0 ? g.w2[1] : g.w2t[0]), H, H);  // next big layer
    epi16<T, 0>(acc, sBias[2 * q + 1], nom, sH2[q], nullptr, nullptr, 0, row0, N);
    __syncthreads();
    float h[4];
    load4(sH2[q] + r * Tile<T>::LD + 4 * lane, h);
    const float v = dot_row(sW3[q], lane, h) + sB3[q];
    if (lane == 0) sq[q][r] = v;
  }
  __syncthreads();
  {
    const float alpha = expf(la);
    float dq[2] = {0.f, 0.f};
    if (n < N) aloss_row(a, sq[0][r], sq[1][r], logp, alpha, n, lane, dq[0], dq[1]);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      T* row = sH2[q] + r * Tile<T>::LD;
      float h[4], d[4];
      load4(row + 4 * lane, h);
      dq_to_dh(dq[q], sW3[q], h, lane, d);
      store4(row + 4 * lane, d);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q) {  // dh1_q in place of h1_q (each element read then written by one lane)
    const f32x4 acc = mma_wf<T, NB>(w2, H, sH2[q]);
    w2 = load_wf<T, NB>((const T*)(q == 0 ? g.w2t[1] : g.aw2t), H, H);
    float m[4];
    tile_mask<T>(sH1[q], m);
    epi16<T, 1>(acc, nullptr, m, sH1[q], nullptr, nullptr, 0, row0, N);
  }
  __syncthreads();
  {
    T* dst = sH2[0] + r * Tile<T>::LD;  // dha2 tile (dh2 no longer needed)
    if (n < N) {
      ahead_row<T>(bb, sH1[0] + r * Tile<T>::LD, sH1[1] + r * Tile<T>::LD, hv, dst, n, lane, sS, sE,
                   r, (size_t)16 * K, sG[r], expf(la));
    } else {
      float z[4] = {0.f, 0.f, 0.f, 0.f};
      store4(dst + 4 * lane, z);
    }
  }
  __syncthreads();
  epi16<T, 1>(mma_wf<T, NB>(w2, H, sH2[0]), nullptr, ha1m, nullptr, nullptr, (T*)g.dha1t, a.ldt, row0, N);
}

}  // namespace sac
