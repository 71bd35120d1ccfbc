// Operand definitions plugged into gemm_rc / gemm_tile / gemm_wg for each layer of the step.
// Output-side ops of gemm_tile split their epilogue into epi(r, c) -- the epilogue's own global
// reads (bias, ReLU mask), issued at the start of the tile so they land under the K loop -- and
// store(r, c, v, e).
// Activations are channels-last (pixel-major, channel-contiguous); frame n = b*T + t
// (batch-major flatten of agents/impala/learning.py:143).
#pragma once
#include "conv1.h"
#include "gemm.h"
#include "lnorm.h"
#include "net.h"

using namespace net;

// conv2: rows oc (64), cols (n, oh, ow) in N*36, k = (kh*4+kw)*32 + ci over act1.
template <typename T> struct Conv2Fwd {
  static constexpr bool A_KMAJOR = false;
  static constexpr bool TILE_EPI = false;
  static constexpr int K = K2;
  int C;
  const T* w;
  const float* b;
  const T* x;
  T* out;
  struct ColCtx { const T* p; };
  DEV ColCtx col_ctx(int c) const {
    const int n = c / P2, p = c - n * P2, oh = p / H2, ow = p - oh * H2;
    return ColCtx{x + ((size_t)(n * H1 + ST2 * oh) * H1 + ST2 * ow) * OC1};
  }
  DEV const T* a_row(int r, int) const { return w + r * K; }
  DEV typename Frag<T>::vec load_b(const ColCtx& cc, int k) const {
    const int tap = k >> 5, ci = k & 31, kh = tap >> 2, kw = tap & 3;
    return Frag<T>::load(cc.p + (kh * H1 + kw) * OC1 + ci);
  }
  struct Epi { float b[4]; };
  DEV Epi epi(int r, int) const { return Epi{{b[r], b[r + 1], b[r + 2], b[r + 3]}}; }
  DEV void store(int r, int c, float v[4], const Epi& e) const {
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = fmaxf(v[i] + e.b[i], 0.f);
    store4(out + (size_t)c * OC2 + r, o);
  }
};

// conv3: rows oc (64), cols (n, oh, ow) in N*16, k = (kh*3+kw)*64 + ci over act2.
// act3 row n is the flattened feature vector in (p*64 + c) order.
template <typename T> struct Conv3Fwd {
  static constexpr bool A_KMAJOR = false;
  static constexpr bool TILE_EPI = false;
  static constexpr int K = K3;
  int C;
  const T* w;
  const float* b;
  const T* x;
  T* out;
  struct ColCtx { const T* p; };
  DEV ColCtx col_ctx(int c) const {
    const int n = c / P3, p = c - n * P3, oh = p / H3, ow = p - oh * H3;
    return ColCtx{x + ((size_t)(n * H2 + oh) * H2 + ow) * OC2};
  }
  DEV const T* a_row(int r, int) const { return w + r * K; }
  DEV typename Frag<T>::vec load_b(const ColCtx& cc, int k) const {
    const int tap = k >> 6, ci = k & 63, kh = tap / 3, kw = tap - kh * 3;
    return Frag<T>::load(cc.p + (kh * H2 + kw) * OC2 + ci);
  }
  struct Epi { float b[4]; };
  DEV Epi epi(int r, int) const { return Epi{{b[r], b[r + 1], b[r + 2], b[r + 3]}}; }
  DEV void store(int r, int c, float v[4], const Epi& e) const {
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = fmaxf(v[i] + e.b[i], 0.f);
    store4(out + (size_t)c * OC3 + r, o);
  }
};

// projection Linear(1024 -> 256) + exact GELU (models/models.py:67-68).
// rows o (256), cols frame n, k = p*64 + c over the LayerNorm output y.
template <typename T> struct FcFwd {
  static constexpr bool A_KMAJOR = false;
  static constexpr bool TILE_EPI = false;
  static constexpr int K = FLAT;
  int C;
  const T* w;
  const float* b;
  const T* y;
  float* zg;  // gelu'(pre-activation), fp32: the GELU backward's factor (head_step phase 3)
  T* h;
  struct ColCtx { const T* p; };
  DEV ColCtx col_ctx(int c) const { return ColCtx{y + (size_t)c * YLD}; }
  DEV const T* a_row(int r, int) const { return w + r * K; }
  DEV typename Frag<T>::vec load_b(const ColCtx& cc, int k) const { return Frag<T>::load(cc.p + k); }
  struct Epi { float b[4]; };
  DEV Epi epi(int r, int) const { return Epi{{b[r], b[r + 1], b[r + 2], b[r + 3]}}; }
  DEV void store(int r, int c, float v[4], const Epi& e) const {
    float gg[4], hh[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) gelu_fwd_grad(v[i] + e.b[i], hh[i], gg[i]);
    store4(zg + (size_t)c * HID + r, gg);
    store4(h + (size_t)c * HID + r, hh);
  }
};

// fp32 FC forward as a split-K GEMM with its combine in the same launch.  The 32 x 32 tile
// kernel (320 workgroups, whole K each) streams 256 KB per workgroup for 1 M MACs and leaves
// 64 CUs with a second tile; here a workgroup owns a 64 (hidden) x 80 (frame) tile over one
// quarter of K: 144 KB streamed for 1.3 M MACs, and 256 workgroups at B*T = 1280 (one per CU).
// Wave w holds rows 16w..16w+15 of the tile as 16 float4 A fragments in registers; the tile's
// 80 frames x 256 k of y sit in LDS.  Each workgroup stores its fp32 partial (20 KB, in the
// accumulator layout) and takes a ticket on its tile's counter; the one that draws the 4th
// ticket sums the four partials in split order ((p0 + p1) + p2) + p3 -- whichever arrives
// last, so the result is deterministic -- and runs FcFwd's bias + GELU epilogue.  Hand-off:
// cdna_hip_programming.md's split-K recipe (plain slab stores, agent release before the
// ticket, agent acquire in the reducer).  The counters only ever grow by 4 per tile per launch
// (zeroed once at create), so no reset is needed.  The 4 splits and the 4 row tiles of a
// column tile run on one XCD when the tile count allows (speed only, not correctness).
namespace fcsk {
constexpr int ROWS = 64, COLS = 80, NS = 4, KS = FLAT / NS, LDB = KS + 4, PART = ROWS * COLS;
constexpr int NCF = COLS / 16, NKB = KS / 16;
}  // namespace fcsk
#if IMPALA_AB  // fc_fwd_splitk_f32 / fc_fwd_wsplit_f32: measured slower, A/B builds only
// PUB (publish form): 1 = write-through (sc1) slab stores and sc1 slab loads, no fences
// (the default); 0 = plain stores, agent release before the ticket, agent acquire in the
// reducer; 2 = measurement knock-out (partials stored, no combine: wrong results).
DEV void st_sc1(float* p, f32x4 v) {
  const unsigned long long lo = __builtin_bit_cast(unsigned long long, float2{v[0], v[1]});
  const unsigned long long hi = __builtin_bit_cast(unsigned long long, float2{v[2], v[3]});
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p) + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV f32x4 ld_sc1(const float* p) {
  auto* q = reinterpret_cast<unsigned long long*>(const_cast<float*>(p));
  const float2 lo = __builtin_bit_cast(float2, __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const float2 hi = __builtin_bit_cast(float2, __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  return f32x4{lo.x, lo.y, hi.x, hi.y};
}
template <int PUB>
__global__ __launch_bounds__(256) void fc_fwd_splitk_f32(const FcFwd<float> op, float* __restrict__ slab,
                                                         unsigned* __restrict__ cnt) {
  using namespace fcsk;
  __shared__ __attribute__((aligned(16))) float sb[COLS * LDB + 4];
  const int nb = (int)gridDim.x, b = (int)blockIdx.x, n_tiles = nb / NS;
  int tile, s;
  if (n_tiles % 8 == 0) {
    const int x = b % 8, l = b / 8;
    tile = x * (n_tiles / 8) + l / NS;
    s = l % NS;
  } else {
    tile = b / NS;
    s = b % NS;
  }
  constexpr int NRT = HID / ROWS;
  const int r0 = (tile % NRT) * ROWS, c0 = (tile / NRT) * COLS, k0 = s * KS;
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // A fragments: row r0 + 16w + (lane & 15), k = k0 + 16 kb + 4 (lane >> 4) + e
  f32x4 a[NKB];
  const float* ap = op.w + (size_t)(r0 + wave * 16 + (lane & 15)) * FLAT + k0 + 4 * (lane >> 4);
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) a[kb] = *reinterpret_cast<const f32x4*>(ap + kb * 16);
  // y tile -> LDS: column (frame) rows of 256 k, padded by 4 floats (conflict-free b128 reads)
#pragma unroll
  for (int i = 0; i < COLS / 4; ++i) {
    const int col = i * 4 + wave, k = lane * 4;
    const int c = min(c0 + col, op.C - 1);  // frames past C: any valid row, results dropped
    *reinterpret_cast<f32x4*>(sb + col * LDB + k) =
        *reinterpret_cast<const f32x4*>(op.y + (size_t)c * YLD + k0 + k);
  }
  __syncthreads();
  f32x4 acc[NCF];
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf) acc[cf] = Frag<float>::zero();
  const float* bp = sb + (lane & 15) * LDB + 4 * (lane >> 4);
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    f32x4 bv[NCF];
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf) bv[cf] = *reinterpret_cast<const f32x4*>(bp + cf * 16 * LDB + kb * 16);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int cf = 0; cf < NCF; ++cf) acc[cf] = Frag<float>::mma_e(e, a[kb], bv[cf], acc[cf]);
  }
  // publish this split's partial, take a ticket
  float* tp = slab + (size_t)tile * NS * PART;
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf) {
    float* dst = tp + (size_t)s * PART + ((wave * NCF + cf) * 64 + lane) * 4;
    if constexpr (PUB == 1) st_sc1(dst, acc[cf]);
    else *reinterpret_cast<f32x4*>(dst) = acc[cf];
  }
  if constexpr (PUB == 2) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* last = reinterpret_cast<int*>(sb + COLS * LDB);
  if (tid == 0) {
    if constexpr (PUB == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned old = __hip_atomic_fetch_add(cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int is_last = (old % NS) == NS - 1;
    if (PUB == 0 && is_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *last = is_last;
  }
  __syncthreads();
  if (!*last) return;
  const int o = r0 + wave * 16 + 4 * (lane >> 4);
  const auto ep = op.epi(o, 0);
  // every partial load of the tile in flight at once (the own split's too: same bits as acc)
  f32x4 p[NCF][NS];
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const float* src = tp + (size_t)q * PART + ((wave * NCF + cf) * 64 + lane) * 4;
      p[cf][q] = PUB == 1 ? ld_sc1(src) : *reinterpret_cast<const f32x4*>(src);
    }
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf) {
    f32x4 v = p[cf][0] + p[cf][1];
#pragma unroll
    for (int q = 2; q < NS; ++q) v += p[cf][q];
    const int c = c0 + cf * 16 + (lane & 15);
    if (c < op.C) {
      float vv[4] = {v[0], v[1], v[2], v[3]};
      op.store(o, c, vv, ep);
    }
  }
}

// fp32 FC forward, K split over the 4 waves of a workgroup instead of over workgroups: a
// workgroup owns 16 hidden x 80 frames over all of K (256 workgroups at B*T = 1280, one per
// CU, 384 KB streamed each against 2 x 256 KB on the CUs that get two 32 x 32 tiles), wave w
// takes k in [256 w, 256 w + 256) with its B fragments straight from global (no operand is
// shared between the waves), and the four 16 x 80 partials meet in LDS, summed in wave order
// ((w0 + w1) + w2) + w3 before FcFwd's bias + GELU epilogue.
namespace fcwk {
constexpr int ROWS = 16, COLS = 80, KW = FLAT / 4, NCF = COLS / 16, NKB = KW / 16, CH = 4;
}  // namespace fcwk
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void fc_fwd_wsplit_f32(
    const FcFwd<float> op) {
  using namespace fcwk;
  __shared__ __attribute__((aligned(16))) float red[4 * NCF * 64 * 4];
  constexpr int NRT = HID / ROWS;
  const int t = xcd_swizzle((int)blockIdx.x, (int)gridDim.x);
  const int r0 = (t % NRT) * ROWS, c0 = (t / NRT) * COLS;
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6, k0 = wave * KW;
  f32x4 a[NKB];
  const float* ap = op.w + (size_t)(r0 + (lane & 15)) * FLAT + k0 + 4 * (lane >> 4);
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) a[kb] = *reinterpret_cast<const f32x4*>(ap + kb * 16);
  const float* bp[NCF];
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf)
    bp[cf] = op.y + (size_t)min(c0 + cf * 16 + (lane & 15), op.C - 1) * YLD + k0 + 4 * (lane >> 4);
  f32x4 acc[NCF];
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf) acc[cf] = Frag<float>::zero();
  // B in chunks of CH k-steps, double-buffered: chunk c + 1 in flight under chunk c's MFMAs
  f32x4 bq[2][CH][NCF];
#pragma unroll
  for (int j = 0; j < CH; ++j)
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf) bq[0][j][cf] = *reinterpret_cast<const f32x4*>(bp[cf] + j * 16);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int ch = 0; ch < NKB / CH; ++ch) {
    if (ch + 1 < NKB / CH) {
#pragma unroll
      for (int j = 0; j < CH; ++j)
#pragma unroll
        for (int cf = 0; cf < NCF; ++cf)
          bq[(ch + 1) & 1][j][cf] = *reinterpret_cast<const f32x4*>(bp[cf] + ((ch + 1) * CH + j) * 16);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the next chunk's loads ahead of these MFMAs
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int cf = 0; cf < NCF; ++cf)
          acc[cf] = Frag<float>::mma_e(e, a[ch * CH + j], bq[ch & 1][j][cf], acc[cf]);
  }
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf)
    *reinterpret_cast<f32x4*>(red + ((wave * NCF + cf) * 64 + lane) * 4) = acc[cf];
  __syncthreads();
  for (int i = tid; i < NCF * 64; i += 256) {
    const int cf = i >> 6, ln = i & 63;
    const float* q = red + (cf * 64 + ln) * 4;
    constexpr int WS = NCF * 64 * 4;  // one wave's partial
    f32x4 v = *reinterpret_cast<const f32x4*>(q) + *reinterpret_cast<const f32x4*>(q + WS);
    v += *reinterpret_cast<const f32x4*>(q + 2 * WS);
    v += *reinterpret_cast<const f32x4*>(q + 3 * WS);
    const int o = r0 + 4 * (ln >> 4), c = c0 + cf * 16 + (ln & 15);
    if (c < op.C) {
      float vv[4] = {v[0], v[1], v[2], v[3]};
      op.store(o, c, vv, op.epi(o, c));
    }
  }
}
#endif  // IMPALA_AB

// actor ‖ critic heads fused into one 16-row GEMM (models/models.py:69-70, 76).
template <typename T> struct HeadsFwd {
  static constexpr bool A_KMAJOR = false;
  static constexpr bool TILE_EPI = false;
  static constexpr int K = HID;
  int C;
  const T* w;
  const float* b;
  const T* h;
  float* out;  // [n][16]: logits 0..A-1, value at 15
  struct ColCtx { const T* p; };
  DEV ColCtx col_ctx(int c) const { return ColCtx{h + (size_t)c * HID}; }
  DEV const T* a_row(int r, int) const { return w + r * K; }
  DEV typename Frag<T>::vec load_b(const ColCtx& cc, int k) const { return Frag<T>::load(cc.p + k); }
  DEV void store(int r, int c, float v[4]) const {
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = v[i] + b[r + i];
    store4(out + (size_t)c * HEADS + r, o);
  }
};

// conv3 + ReLU + LayerNorm(1024) fused (models/common.py:117-119, models/models.py:66):
// a 64(oc) x 64(pixel) tile holds 4 whole frames; wave w normalises frame w of the tile.
// Writes act3 (post-ReLU, kept for the mask and the LN backward), y = LN(act3), mean/rstd.
template <typename T> struct Conv3LnFwd : Conv3Fwd<T> {
  static constexpr bool TILE_EPI = true;
  const float* gam;  // permuted to p*64 + c
  const float* bet;
  T* y;
  float* stats;
  int frames_per_tile;  // tile width / 16 (<= 4: one wave per frame)
  typedef LnLane EpiConst;  // loaded once per workgroup (gemm_tile)
  DEV EpiConst epi_const(int tid) const { return ln_lane_consts(tid & 63, this->b, gam, bet); }
  DEV void tile_epilogue(const float* et, int ldt, int, int cc0, int tid,
                         const EpiConst& k) const {
    const int lane = tid & 63, wave = tid >> 6;
    const int frame = cc0 / P3 + wave;
    if (wave >= frames_per_tile || (frame + 1) * P3 > this->C) return;
    ln_frame_epilogue<T>(et + wave * P3 * ldt, ldt, frame, lane, k, this->out, y, stats);
  }
};

// dy = dz . Wfc  (rows j in p*64+c order, cols frame), fp32 out for the LayerNorm backward.
// A[j][o] = wfc[o][j]: read k-major from the forward weight (no transposed copy).
template <typename T> struct FcDgrad {
  static constexpr bool A_KMAJOR = true;
  static constexpr bool TILE_EPI = false;
  static constexpr int K = HID;
  int C;
  const T* w;   // wfc [256][1024]
  const T* dz;
  float* dy;
  struct ColCtx { const T* p; };
  DEV ColCtx col_ctx(int c) const { return ColCtx{dz + (size_t)c * HID}; }
  DEV const T* a_row(int, int) const { return nullptr; }
  DEV const T* a_kptr(int k, int r, int) const { return w + (size_t)k * FLAT + r; }
  DEV typename Frag<T>::vec load_b(const ColCtx& cc, int k) const { return Frag<T>::load(cc.p + k); }
  struct Epi {};
  DEV Epi epi(int, int) const { return Epi{}; }
  DEV void store(int r, int c, float v[4], const Epi&) const { store4(dy + (size_t)c * FLAT + r, v); }
};

// conv3 dgrad (gather form): rows ci (64), cols input pixel (n, iy, ix) in N*36,
// k = (kh*3+kw)*64 + oc; B = dact3[n][iy-kh][ix-kw][oc] (0 outside the 4x4 output).
// Epilogue applies conv2's ReLU mask (act2 > 0).
template <typename T> struct Conv3Dgrad {
  static constexpr bool A_KMAJOR = true;
  static constexpr bool TILE_EPI = false;
  static constexpr int K = K3;
  int C;
  const T* w;     // w3 [64 oc][576 = tap*64 + ci]; A[ci][tap*64 + oc] read k-major
  const T* dy;    // dact3 [n][16][64]
  const T* act;   // act2 (mask)
  T* dx;          // dact2
  struct ColCtx { const T* p; int iy, ix; };
  DEV ColCtx col_ctx(int c) const {
    const int n = c / P2, p = c - n * P2, iy = p / H2, ix = p - iy * H2;
    return ColCtx{dy + (size_t)n * P3 * OC3, iy, ix};
  }
  DEV const T* a_row(int, int) const { return nullptr; }
  DEV const T* a_kptr(int k, int r, int) const {
    const int tap = k >> 6, oc = k & 63;
    return w + (size_t)oc * K3 + tap * OC2 + r;
  }
  DEV typename Frag<T>::vec load_b(const ColCtx& cc, int k) const {
    const int tap = k >> 6, oc = k & 63, kh = tap / 3, kw = tap - kh * 3;
    const int oy = cc.iy - kh, ox = cc.ix - kw;
    if (oy < 0 || oy >= H3 || ox < 0 || ox >= H3) return Frag<T>::zero();
    return Frag<T>::load(cc.p + (oy * H3 + ox) * OC3 + oc);
  }
  struct Epi { float a[4]; };  // act2 at the output position (conv2's ReLU mask)
  DEV Epi epi(int r, int c) const {
    Epi e;
    load4(act + (size_t)c * OC2 + r, e.a);
    return e;
  }
  DEV void store(int r, int c, float v[4], const Epi& e) const {
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = e.a[i] > 0.f ? v[i] : 0.f;
    store4(dx + (size_t)c * OC2 + r, o);
  }
};

template <typename T> struct FcWgrad {  // dWfc[o][j] = sum_n dz[n][o] y[n][j]
  static constexpr int R = HID, C = FLAT;
  int M;
  float out_scale = 1.f;
  const T* x;  // dz
  int x_ld = HID;
  const T* y;
  // Y gather as element offsets from y (buffer loads: out-of-range rows read as zero)
  DEV int y_roff(int m) const { return m * YLD; }
  DEV int y_coff(int c) const { return c; }
  DEV int y_bytes() const { return M * YLD * (int)sizeof(T); }
  DEV const T* ybase() const { return y; }
};
// The FC weight gradient over the whole batch in one split (gemm_wg direct mode): the tile is
// final, so it is written straight into the canonical gradient (o*1024 + c*16 + p for kernel
// column j = p*64 + c; the bias into bfc) and the workgroup's sum of squares goes to its own
// clip-norm partial slot -- no fp32 partial slab and no reduction pass for this layer.
template <typename T> struct FcWgradDirect : FcWgrad<T> {
  static constexpr bool DIRECT = true;
  float* grads;       // canonical gradient buffer
  long long wcanon;   // canonical offset of wfc (bfc follows at wcanon + HID * FLAT)
  float* sumsq;       // [workgroups] partial sums of squares
  DEV long long canon(int o, int j) const {
    return wcanon + (long long)o * FLAT + (j & 63) * 16 + (j >> 6);
  }
  DEV long long bias_canon(int o) const { return wcanon + (long long)HID * FLAT + o; }
};

template <typename T> struct Conv3Wgrad {  // m = (n, oy, ox) in N*16; c = (kh*3+kw)*64 + ci
  static constexpr int R = OC3, C = K3;
  int M;
  float out_scale = 1.f;
  const T* x;  // dact3
  int x_ld = OC3;
  const T* in;  // act2
  DEV int y_roff(int m) const {  // top-left input pixel of the 3x3 patch
    const int n = m / P3, p = m - n * P3, oy = p / H3, ox = p - oy * H3;
    return ((n * H2 + oy) * H2 + ox) * OC2;
  }
  DEV int y_coff(int c) const {
    const int tap = c >> 6, ci = c & 63, kh = tap / 3, kw = tap - kh * 3;
    return (kh * H2 + kw) * OC2 + ci;
  }
  DEV int y_bytes() const { return (M / P3) * (H2 * H2 * OC2) * (int)sizeof(T); }
  DEV const T* ybase() const { return in; }
  // row cursor (gemm_wg_body YCUR): (frame, pixel) of row m, advanced by a chunk stride without
  // the divisions of y_roff (which the compiler also put behind a branch per staging load)
  static constexpr bool YCUR = true;
  struct YCur { int n, p; };
  DEV YCur ycur(int m) const { const int n = m / P3; return YCur{n, m - n * P3}; }
  template <int D> DEV void ycur_adv(YCur& c) const {
    c.p += D % P3;
    c.n += D / P3;
    if (c.p >= P3) { c.p -= P3; c.n += 1; }
  }
  DEV int ycur_off(const YCur& c) const {
    const int oy = c.p / H3, ox = c.p - oy * H3;
    return ((c.n * H2 + oy) * H2 + ox) * OC2;
  }
};
template <typename T> struct Conv2Wgrad {  // m = (n, oy, ox) in N*36; c = (kh*4+kw)*32 + ci
  static constexpr int R = OC2, C = K2;
  int M;
  float out_scale = 1.f;
  const T* x;  // dact2
  int x_ld = OC2;
  const T* in;  // act1
  DEV int y_roff(int m) const {
    const int n = m / P2, p = m - n * P2, oy = p / H2, ox = p - oy * H2;
    return ((n * H1 + ST2 * oy) * H1 + ST2 * ox) * OC1;
  }
  DEV int y_coff(int c) const {
    const int tap = c >> 5, ci = c & 31, kh = tap >> 2, kw = tap & 3;
    return (kh * H1 + kw) * OC1 + ci;
  }
  DEV int y_bytes() const { return (M / P2) * (H1 * H1 * OC1) * (int)sizeof(T); }
  DEV const T* ybase() const { return in; }
  static constexpr bool YCUR = true;  // see Conv3Wgrad
  struct YCur { int n, p; };
  DEV YCur ycur(int m) const { const int n = m / P2; return YCur{n, m - n * P2}; }
  template <int D> DEV void ycur_adv(YCur& c) const {
    c.p += D % P2;
    c.n += D / P2;
    if (c.p >= P2) { c.p -= P2; c.n += 1; }
  }
  DEV int ycur_off(const YCur& c) const {
    const int oy = c.p / H2, ox = c.p - oy * H2;
    return ((c.n * H1 + ST2 * oy) * H1 + ST2 * ox) * OC1;
  }
};

// FC weight gradient and FC input gradient in ONE launch.  Both read only dz (with y / Wfc), so
// they are independent: blocks [0, gx*gy*gz) run the split weight-gradient body (gemm_wg, G
// 4-wave groups) and the rest run the input-gradient tiles (gemm_tile with 4*G waves: 64 x 64
// tiles for G = 1, 128 x 64 for G = 2).  The weight gradient's 96 workgroups leave most CUs
// idle for its ~7 us; the dgrad tiles fill them instead of running after it.  Same per-tile
// arithmetic as the two separate kernels (same tile shapes for the weight gradient).
// dgrad tiles DR (flat) x DC (frames) on DWR x DWC waves, weight-gradient tiles 64 x WBC.
// fp32: 64 x 80 dgrad tiles (256 at N = 1280, 78 KB of LDS) beside 256 weight-gradient
// workgroups of 64 x 128 (the same 8 splits, 51 KB): 512 workgroups of about the same MFMA
// work, two per CU -- two waves per SIMD (profiles/r05kw: 64 x 64 dgrad tiles beside 64 x 256
// weight-gradient tiles ran ~1.75 rounds at one workgroup per CU, 20.6 us; 128 x 80 one round
// at one per CU, 19.7; this 16.7)
// bf16 (G = 2, 8 waves): 64 x 64 dgrad tiles on 2 x 4 waves (320) beside 64 x 128 weight-gradient
// workgroups (192 at the same 6 splits), 78 KB: 512 workgroups, two per CU (8.4 -> 6.8 us)
constexpr int FCB_DR32 = 64, FCB_DC32 = 80, FCB_DWR32 = 4, FCB_DWC32 = 1;
constexpr int FCB_WBC32 = 128;
template <typename T, int G> struct FcBwdCfg {
  static constexpr int DR = G == 2 ? 64 : FCB_DR32, DWR = G == 2 ? 2 : FCB_DWR32;
  static constexpr int DC = G == 2 ? 64 : FCB_DC32, DWC = G == 2 ? 4 : FCB_DWC32;
  static constexpr int DBK = sizeof(T) == 2 ? 128 : 64;
  static constexpr int WBC = G == 2 ? 128 : FCB_WBC32;
  static constexpr int SW = gemm_wg_smem<T, 64, WBC, 32, G>();
  static constexpr int SD = gemm_tile_smem<T, DR, DC, DBK, DWR, DWC, FcDgrad<T>>();
  static constexpr int SMEM = SW > SD ? SW : SD;
};
template <typename T, int G>
__global__ __launch_bounds__(256 * G) void fc_bwd_kernel(const FcWgrad<T> ow, float* __restrict__ slab,
                                                         float* __restrict__ slab_bias, int mps,
                                                         int gx, int gy, int gz,
                                                         const FcDgrad<T> od, int n_rtiles) {
  using C = FcBwdCfg<T, G>;
  __shared__ __attribute__((aligned(16))) T smem[C::SMEM];
  const int nw = gx * gy * gz;
  if ((int)blockIdx.x < nw)
    gemm_wg_body<T, 64, C::WBC, 1, 4, 32, G, FcWgrad<T>>(ow, slab, slab_bias, mps, (int)blockIdx.x,
                                                         gx, gy, gz, smem);
  else
    gemm_tile_body<T, C::DR, C::DC, C::DBK, C::DWR, C::DWC, FcDgrad<T>>(od, n_rtiles, (int)blockIdx.x - nw,
                                                                (int)gridDim.x - nw, smem);
}

// conv3 and conv2 weight gradients in ONE launch (both depend only on the LayerNorm backward's
// outputs): blocks [0, n3) run the conv3 split weight-gradient body, the rest conv2's -- the
// same tiles, splits and group order as the two separate launches (bitwise-equal slabs), with
// one kernel boundary fewer and conv3's tail overlapping conv2's ramp.
// conv2 weight-gradient tile of the merged launch: fp32 64 x 64 on 2 x 2 waves -- 512 workgroups
// of conv3's size (64 splits as before, so the same slab and per-element sums), three per CU
// beside conv3's 252, instead of 256 64 x 128 workgroups of twice conv3's MFMA work; bf16 64 x 128
template <typename T> struct Wg2Tile {
  static constexpr int BC = sizeof(T) == 4 ? 64 : 128, WR = sizeof(T) == 4 ? 2 : 1, WC = 4 / WR;
};
template <typename T, int G> struct Wg23Cfg {
  static constexpr int S3 = gemm_wg_smem<T, 64, 64, 32, G>(), S2 = gemm_wg_smem<T, 64, Wg2Tile<T>::BC, 32, G>();
  static constexpr int SMEM = S3 > S2 ? S3 : S2;
};
template <typename T, int G>
__global__ __launch_bounds__(256 * G) void wgrad23_kernel(const Conv3Wgrad<T> o3, float* __restrict__ s_w3,
                                                          float* __restrict__ s_b3, int mps3, int g3x, int g3z,
                                                          const Conv2Wgrad<T> o2, float* __restrict__ s_w2,
                                                          float* __restrict__ s_b2, int mps2, int g2x, int g2z) {
  __shared__ __attribute__((aligned(16))) T smem[Wg23Cfg<T, G>::SMEM];
  const int n3 = g3x * g3z;
  if ((int)blockIdx.x < n3)
    gemm_wg_body<T, 64, 64, 2, 2, 32, G, Conv3Wgrad<T>>(o3, s_w3, s_b3, mps3, (int)blockIdx.x, g3x, 1,
                                                        g3z, smem);
  else
    gemm_wg_body<T, 64, Wg2Tile<T>::BC, Wg2Tile<T>::WR, Wg2Tile<T>::WC, 32, G, Conv2Wgrad<T>>(
        o2, s_w2, s_b2, mps2, (int)blockIdx.x - n3, g2x, 1, g2z, smem);
}

#if IMPALA_AB  // fwd_chain_kernel: measured slower, A/B builds only
// The trunk forward and the FC forward in ONE launch (bf16, conv3 tail on): blocks [0, n_conv)
// run the per-frame conv1 / conv2 / conv3+LayerNorm body and publish a flag each; the FC tile
// blocks after them (64 hidden units x 32 frames, 8 waves, one tile per block) wait only for
// the conv blocks that produce their 32 frames of y, then run the FC body.  Hand-off
// (MI355X_MICROARCH.md, inter-workgroup visibility, R1): the producer stores y write-through
// (sc1), every storing wave drains, and one lane stores flag = epoch (relaxed, agent); the
// consumer polls relaxed, acquires at agent scope once, then a barrier, then plain loads.  The FC blocks are dispatched after every
// conv block, so a waiting block never holds a slot a producer needs; the poll is bounded (a
// timeout sets *fault and continues).  epoch changes every launch (never 0).
template <typename T> struct FwdChainCfg {
  static constexpr int FR = 64, FC = 32, FK = 256, FWR = 4, FWC = 2;  // FC tile, 8 waves
  static constexpr int SD = gemm_tile_smem<T, FR, FC, FK, FWR, FWC, FcFwd<T>>();
  static constexpr int SMEM = C12FLds<T>::ELEMS > SD ? C12FLds<T>::ELEMS : SD;
};
template <typename T>
__global__ __launch_bounds__(512) void fwd_chain_kernel(
    const uint8_t* __restrict__ x, const T* __restrict__ w1, const float* __restrict__ b1,
    const T* __restrict__ w2, const float* __restrict__ b2, T* __restrict__ act1,
    uint32_t* __restrict__ mask, T* __restrict__ act2, int N, int fpw, const C3Tail<T> c3,
    int n_conv, const FcFwd<T> fc, unsigned* __restrict__ flags, unsigned epoch,
    unsigned* __restrict__ fault) {
  static_assert(c12f_groups<T>() == 2, "512-thread conv body (bf16)");
  using C = FwdChainCfg<T>;
  __shared__ __attribute__((aligned(16))) T smem[C::SMEM];
  const int b = (int)blockIdx.x;
  if (b < n_conv) {
    // y is the only payload the FC blocks read; c3.y_sc1 stores it write-through, so the
    // publish is: every storing wave drains, a barrier, one lane stores the flag (R1)
    conv12_fwd_body<T>(x, w1, b1, w2, b2, act1, mask, act2, N, fpw, c3, b, smem);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store(flags + b, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // FC tile of this block (gemm_tile_body's tile order: row tile fastest)
  const int vb = b - n_conv, vg = (int)gridDim.x - n_conv;
  const int n_rt = HID / C::FR;
  const int t = xcd_swizzle(vb, vg);
  const int c0 = (t / n_rt) * C::FC;
  if (threadIdx.x < 64) {  // wave 0: lane i polls producer p0 + i
    const int p0 = c0 / fpw, p1 = (min(N, c0 + C::FC) - 1) / fpw;
    const int p = p0 + (int)threadIdx.x;
    bool ok = p > p1 ||
              __hip_atomic_load(flags + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
    for (unsigned spins = 0; !__all(ok); ++spins) {
      if (spins > (1u << 22)) {  // ~0.1 s: a producer never finished; do not hang the GPU
        if (threadIdx.x == 0) __hip_atomic_store(fault, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
      ok = ok || __hip_atomic_load(flags + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
    }
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  gemm_tile_body<T, C::FR, C::FC, C::FK, C::FWR, C::FWC, FcFwd<T>>(fc, n_rt, vb, vg, smem);
}
#endif  // IMPALA_AB
