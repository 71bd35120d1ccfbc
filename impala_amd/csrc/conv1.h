// conv1 (Conv2d(3, 32, 8, stride 4) on u8 64x64 frames, models/common.py:113-114) as a
// space-to-depth 2x2 stride-1 convolution, forward and weight gradient.
//
//   x[ci][4Y+b][4X+d]  ->  s2d[Y][X][ch],  ch = ci*16 + b*4 + d  (48 channels, 16x16 grid)
//   kh = 4a + b, kw = 4c + d  ->  tap = a*2 + c,  k' = tap*48 + ch   (K = 192)
//   out[oy][ox][oc] = sum_{tap, ch} W'[oc][k'] * s2d[oy+a][ox+c][ch]
//
// A workgroup loops over whole frames: the frame's 12 KB of bytes are loaded with coalesced
// 16-byte loads (one frame ahead, in registers), converted to the compute type ONCE per byte
// and scattered into an LDS s2d image whose rows (one per grid cell) are padded to a
// bank-conflict-free stride.  The im2col is then only addressing: every MFMA B fragment is a
// per-lane LDS read at row(pixel, tap) -- ds_read_b128 for the forward, the transposing
// ds_read_b64_tr_b16 (bf16) for the weight gradient, where the reduction runs over pixels.
#pragma once
#include "gemm.h"
#include "lnorm.h"
#include "net.h"

using namespace net;

namespace c1 {
constexpr int GRID = 16;                 // 16x16 super-pixels of 4x4
constexpr int CH = 48;                   // 3 * 4 * 4
constexpr int NPIX = P1;                 // 225 output pixels per frame
constexpr int NPAD = 256;                // pixels padded to a multiple of 32 (wgrad k-steps)
template <typename T> struct L;
template <> struct L<__bf16> { static constexpr int LDI = 56; };  // 112 B rows: conflict-free
template <> struct L<float> { static constexpr int LDI = 52; };
}  // namespace c1

// Fused forward image layout: row-major s2d rows of LDI_F elements, GRID*GRID + 2 rows (the
// conv1 pixel tiles are grid rows oy with lane = ox in 0..15, ox = 15 a pad column, whose taps
// reach row 256).  With grid-indexed tiles the 16 lanes of a B fragment read 16 consecutive
// rows, so 96-byte rows (bf16, no padding) make every ds_read_b128 conflict-free
// (tools/ldsbank.py: 1.00x, against 2.80x for pixel-indexed tiles on 112-byte rows).
// Backward (conv12_bwd) tile pitches, from tools/ldsbank.py: s2d image rows of 52 bf16 (frame
// stash 1.00x vs 2.00x at 56), dY1 rows of 36 (its masked stores 1.88x vs 3.75x at 40), dY2
// cell rows of 80 (its ds_read_b128 2.00x vs 3.00x at 72)
namespace c1 {
template <typename T> struct LB;
template <> struct LB<__bf16> { static constexpr int LDI = 52, LDX = 36, LD2 = 80; };
template <> struct LB<float> { static constexpr int LDI = 52, LDX = 36, LD2 = 68; };
template <typename T> struct LF;
template <> struct LF<__bf16> { static constexpr int LDI = 48; };
template <> struct LF<float> { static constexpr int LDI = 52; };
constexpr int FROWS = GRID * GRID + 2;
}  // namespace c1

// canonical conv1 weight index (oc, ci, kh, kw) <-> s2d kernel order k'
DEV int c1_kprime(int ci, int kh, int kw) {
  return ((kh >> 2) * 2 + (kw >> 2)) * c1::CH + ci * 16 + (kh & 3) * 4 + (kw & 3);
}
DEV int c1_canon_k(int kp) {  // k' -> ci*64 + kh*8 + kw
  const int tap = kp / c1::CH, ch = kp - tap * c1::CH;
  const int ci = ch >> 4, b = (ch >> 2) & 3, d = ch & 3;
  return ci * 64 + ((tap >> 1) * 4 + b) * 8 + (tap & 1) * 4 + d;
}

// LDS row (grid cell) of output pixel p under tap (a, c)
DEV int c1_row(int p, int tap) {
  const int oy = p / H1, ox = p - oy * H1;
  return (oy + (tap >> 1)) * c1::GRID + ox + (tap & 1);
}

// frame bytes -> LDS s2d image.  Thread t owns 16-byte vectors t, t+256, t+512 of the frame.
template <typename T>
DEV void c1_load_frame(const uint8_t* __restrict__ frame, int tid, uint4 v[3]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) v[i] = reinterpret_cast<const uint4*>(frame)[tid + i * 256];
}
// Which row of the batch arrays holds frame f.  ObsDirect: row f.  ObsRows
// (impala_train_step_rows): the arrays are a replay ring read in place -- trajectory b of the
// batch is ring slot rows[b], so frame f = b * T + t is ring row rows[b] * T + t (the same map
// serves the per-frame actions, rewards, discounts and logits in head_step_kernel).  The map is
// the kernels' last argument (dynamic indexing of a by-value kernel argument is a load from the
// argument segment); ObsDirect is empty, so the other arguments keep their offsets.
constexpr int kObsRowsMax = 256;
struct ObsDirect {  // (empty: the identity map)
  DEV size_t map(size_t f) const { return f; }
};
struct ObsRows {
  int T;
  int rows[kObsRowsMax];
  DEV size_t map(size_t f) const {
    const int b = (int)(f / (size_t)T);
    return (size_t)rows[b] * (size_t)T + (f - (size_t)b * (size_t)T);
  }
};

template <typename T, int LDI = c1::L<T>::LDI>
DEV void c1_stash_frame(T* img, int tid, const uint4 v[3]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int vi = tid + i * 256, ci = vi >> 8, yy = (vi & 255) >> 2, xq = vi & 3;
    const int Y = yy >> 2, b = yy & 3;
    const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // 4 bytes = d 0..3 of grid column X = 4*xq + q
      T* dst = img + (Y * c1::GRID + 4 * xq + q) * LDI + ci * 16 + b * 4;
      const uint32_t u = w[q];
      if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<f32x4*>(dst) = f32x4{(float)(u & 255u), (float)((u >> 8) & 255u),
                                               (float)((u >> 16) & 255u), (float)(u >> 24)};
      } else {
        bf16x4 o;
        o[0] = (__bf16)(float)(u & 255u);
        o[1] = (__bf16)(float)((u >> 8) & 255u);
        o[2] = (__bf16)(float)((u >> 16) & 255u);
        o[3] = (__bf16)(float)(u >> 24);
        *reinterpret_cast<bf16x4*>(dst) = o;
      }
    }
  }
}

// frame bytes -> row-major s2d image of LDI-element rows, the four 8-byte (bf16) / 16-byte
// (fp32) pieces of a lane's vector written in the rotated order q = (j + xq) & 3: the 16 lanes
// of a store group then hit 16 different bank pairs (tools/ldsbank.py stash_rot: 1.00x; the
// plain order is 4x on 96-byte rows)
template <typename T, int LDI>
DEV void c1_stash_frame_rot(T* img, int tid, const uint4 v[3]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int vi = tid + i * 256, ci = vi >> 8, yy = (vi & 255) >> 2, xq = vi & 3;
    const int Y = yy >> 2, b = yy & 3;
    const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = (j + xq) & 3;
      // word q selected with masks: the nested select compiled to a divergent branch per
      // value of q (12 x 4 exec-masked blocks, 1.7-2.2k clocks per frame; fwdstash32 r04v4)
      const uint32_t u = (w[0] & -(uint32_t)(q == 0)) | (w[1] & -(uint32_t)(q == 1)) |
                         (w[2] & -(uint32_t)(q == 2)) | (w[3] & -(uint32_t)(q == 3));
      T* dst = img + (Y * c1::GRID + 4 * xq + q) * LDI + ci * 16 + b * 4;
      if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<f32x4*>(dst) = f32x4{(float)(u & 255u), (float)((u >> 8) & 255u),
                                               (float)((u >> 16) & 255u), (float)(u >> 24)};
      } else {
        bf16x4 o;
        o[0] = (__bf16)(float)(u & 255u);
        o[1] = (__bf16)(float)((u >> 8) & 255u);
        o[2] = (__bf16)(float)((u >> 16) & 255u);
        o[3] = (__bf16)(float)(u >> 24);
        *reinterpret_cast<bf16x4*>(dst) = o;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// forward: act1[n][p][oc] = relu(sum W'[oc][k'] s2d * 1/255 + b1), weights in registers;
// optionally the ReLU bit mask mask[n][p] (bit oc = act1 > 0) for the fused backward.
// ---------------------------------------------------------------------------------------
// W1 as bf16 conv1 A fragments (bf16 fragment layout: 8 consecutive k per lane), rows
// oc = 16 i + (lane & 15): bf16 W1 as is; fp32 W1 split exactly into three bf16 terms
// x = hi + mid + lo (round-to-nearest 8-bit pieces of a 24-bit significand: every product with
// an image byte, exact in bf16, is exact in the fp32 accumulator, so the three MFMA passes
// compute the fp32 products).  Shared by both conv1 forward kernels (bitwise-equal act1).
DEV void c1_split3(float x, __bf16& h, __bf16& m, __bf16& l) { split3(x, h, m, l); }
// fp32 W1 staged once per workgroup as its three bf16 planes (plane p: [32][C1W_LD] bf16, rows
// padded by 16: conflict-free 16-byte fragment reads), instead of every wave loading all of W1
// (4 x 24.6 KB through the CU's load path) and splitting it
constexpr int C1W_LD = K1 + 16;
DEV void c1_stage_w1_f32(const float* __restrict__ w1, __bf16* __restrict__ planes, int tid) {
  constexpr int NV = OC1 * K1 / 4;  // float4s
#pragma unroll
  for (int i = 0; i < NV / 256; ++i) {
    const int e = tid + 256 * i, r = e / (K1 / 4), c = (e % (K1 / 4)) * 4;
    const f32x4 u = *reinterpret_cast<const f32x4*>(w1 + (size_t)e * 4);
    bf16x4 o[3];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __bf16 h, m, l;
      c1_split3(u[q], h, m, l);
      o[0][q] = h;
      o[1][q] = m;
      o[2][q] = l;
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<bf16x4*>(planes + (p * OC1 + r) * C1W_LD + c) = o[p];
  }
}

template <typename T>
DEV void c1_load_w1(const T* __restrict__ w1, int lane,
                    Frag<__bf16>::vec (&wa)[2][K1 / Frag<__bf16>::KSTEP][sizeof(T) == 4 ? 3 : 1]) {
  using FB = Frag<__bf16>;
  constexpr int NKB = K1 / FB::KSTEP;
  const int klb = FB::KPL * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      const T* src = w1 + (16 * i + (lane & 15)) * K1 + kb * FB::KSTEP + klb;
      if constexpr (sizeof(T) == 2) {
        wa[i][kb][0] = FB::load(src);
      } else {
        const f32x4 u0 = *reinterpret_cast<const f32x4*>(src), u1 = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          __bf16 h, m, l;
          c1_split3(c < 4 ? u0[c] : u1[c - 4], h, m, l);
          wa[i][kb][0][c] = h;
          wa[i][kb][1][c] = m;
          wa[i][kb][2][c] = l;
        }
      }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void conv1_fwd_s2d(const uint8_t* __restrict__ x,
                                                     const T* __restrict__ w,  // [32][192] k'
                                                     const float* __restrict__ bias,
                                                     T* __restrict__ out,
                                                     uint32_t* __restrict__ mask, int N) {
  // the image in LDS as bf16 (exact bytes) in both modes; conv1 on bf16 MFMAs (fp32: three
  // exact passes, c1_load_w1)
  using FB = Frag<__bf16>;
  typedef FB::vec VB;
  constexpr int LDI = c1::L<__bf16>::LDI;
  constexpr int NKB = K1 / FB::KSTEP, NT = sizeof(T) == 4 ? 3 : 1;
  __shared__ __attribute__((aligned(16))) __bf16 img[c1::GRID * c1::GRID * LDI];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kl = FB::KPL * (lane >> 4);
  VB wa[2][NKB][NT];  // A fragments: rows oc = 16*i + (lane & 15), all of K
  c1_load_w1<T>(w, lane, wa);
  float bb[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) bb[i][q] = bias[16 * i + 4 * (lane >> 4) + q];
  int f = blockIdx.x;
  if (f >= N) return;
  uint4 nv[3];
  c1_load_frame<T>(x + (size_t)f * IMG, tid, nv);
  for (; f < N; f += gridDim.x) {
    __syncthreads();  // previous frame's readers are done
    c1_stash_frame<__bf16>(img, tid, nv);
    __syncthreads();
    if (f + (int)gridDim.x < N) c1_load_frame<T>(x + (size_t)(f + gridDim.x) * IMG, tid, nv);
    for (int tile = wave; tile < 15; tile += 4) {  // 15 x 16 pixel tiles cover the 225 pixels
      const int p = min(tile * 16 + (lane & 15), c1::NPIX - 1);
      const int base = c1_row(p, 0) * LDI;
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        const int k = kb * FB::KSTEP + kl, tap = k / c1::CH, ch = k - tap * c1::CH;
        const int off = ((tap >> 1) * c1::GRID + (tap & 1)) * LDI + ch;
        const VB b = *reinterpret_cast<const VB*>(img + base + off);
#pragma unroll
        for (int tm = 0; tm < NT; ++tm) {
          acc[0] = FB::mma(wa[0][kb][tm], b, acc[0]);
          acc[1] = FB::mma(wa[1][kb][tm], b, acc[1]);
        }
      }
      const int pc = tile * 16 + (lane & 15);
      uint32_t bits = 0;  // ReLU mask of this pixel's 32 channels (bit oc), for the backward
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = fmaxf(acc[i][q] * (1.f / 255.f) + bb[i][q], 0.f);
          bits |= (v[q] > 0.f ? 1u : 0u) << (16 * i + 4 * (lane >> 4) + q);
        }
        if (pc < c1::NPIX) store4(out + ((size_t)f * c1::NPIX + pc) * OC1 + 16 * i + 4 * (lane >> 4), v);
      }
      bits = xor32_or(xor16_or(bits));
      if (mask && pc < c1::NPIX && lane < 16) mask[(size_t)f * c1::NPIX + pc] = bits;
    }
  }
}

// ---------------------------------------------------------------------------------------
// conv1 + conv2 forward, fused per frame: the frame's act1 (15x15x32) is produced into LDS and
// consumed there by conv2 (it is also written to HBM, with its ReLU bit mask, for the backward).
//   conv1: as conv1_fwd_s2d (weights in registers, 15 pixel tiles over the 4 waves)
//   conv2: act2[p][oc] = relu(sum_k W2[oc][k] act1[2oy+kh][2ox+kw][ci] + b2), k = tap*32 + ci;
//          wave w owns oc tile w (its W2 rows stay in registers), 3 tiles of 16 output pixels,
//          B fragments are 16-byte LDS reads of the act1 tile (one tap per 32-wide k-step).
// G 4-wave groups per workgroup take alternating frames of the workgroup's run.
// ---------------------------------------------------------------------------------------
template <typename T> constexpr int c12f_groups() { return sizeof(T) == 2 ? 2 : 1; }
// waves per frame group: fp32 runs one frame at a time (its act1 tile and the frames' act2 fill
// the LDS) on 8 waves, two per SIMD.  wq = wave & 3 takes the conv1 row phase and the conv2 /
// conv3 output-channel tile, wh = wave >> 2 the conv1 output-channel tile.  conv2 and the conv3
// GEMM run on waves 0..3 as before (split further, every wave would stream the W2 rows of its
// tile: twice the weight traffic, 60 -> 68 us, profiles/r05fw8); waves 4..7 stash the next
// image under waves 0..3's conv2.  Each output's k order is the 4-wave one (bitwise equal).
template <typename T> constexpr int c12f_wpg() { return sizeof(T) == 2 ? 4 : 8; }
template <typename T> constexpr int c12f_threads() { return 64 * c12f_wpg<T>() * c12f_groups<T>(); }

// Optional conv3 + ReLU + LayerNorm tail of the fused forward (bf16): after its frames, the
// workgroup stages W3 in LDS and computes conv3 for them from act2 kept in LDS, one wave per
// frame, with the same k-step order and fragment layout as gemm_tile<Conv3LnFwd> and the same
// ln_frame_epilogue, so act3 / y / stats are bit-identical to the separate conv3 launch.
constexpr int C3T_FMAX = 6;  // frames per workgroup the tail supports (wave per frame, LDS)
// fp32: the frames' act2 tiles (36 cells of 68 floats each) fit beside the image and the act1
// tile for at most 5 frames (C2's run: 1280 frames / 256 workgroups)
template <typename T> constexpr int c3t_fmax() { return sizeof(T) == 2 ? C3T_FMAX : 5; }
template <typename T> struct C3Tail {
  const T* w3;       // kernel-layout W3 [64][576 = tap*64 + ci]
  const float* b3;
  const float* gam;  // LayerNorm gamma / beta, p*64+c order
  const float* bet;
  T* act3;           // nullptr: no tail (the separate conv3 launch runs)
  T* y;
  float* stats;
  int y_sc1;         // y stored write-through (read by other workgroups of the same launch)
};

// LDS of the forward body (elements of T)
template <typename T> struct C12FLds {
  static constexpr int VEC = 16 / (int)sizeof(T), LDA1 = OC1 + VEC, A1P = 22;
  static constexpr int IMGSZ = c1::FROWS * c1::LF<T>::LDI, GSZ = IMGSZ + A1P * 16 * LDA1;
  static constexpr int LDA2 = OC2 + VEC;
  // act2 tile rows: bf16 6 x 7 cells (one pad column), fp32 6 x 6 (the LDS budget)
  static constexpr int A2W = sizeof(T) == 2 ? H2 + 1 : H2;
  static constexpr int A2SZ = c3t_fmax<T>() * H2 * A2W * LDA2;
  // bf16: the W2 staging rows from group 1's act1 tile on (W1 in group 0's), past the act2 tiles
  static constexpr int WSTG = sizeof(T) == 2 ? GSZ + IMGSZ + OC2 * (K2 + 2 * VEC) : 0;
  static constexpr int ELEMS = c12f_groups<T>() * GSZ + A2SZ > WSTG ? c12f_groups<T>() * GSZ + A2SZ : WSTG;
};

// The kernel body on workgroup `wg` (frames wg*fpw ..) with the LDS passed in
// (C12FLds<T>::ELEMS elements)
// act1's store cache policy: bf16 streams it non-temporally (nt: it is re-read only by the
// conv2 weight gradient two launches later), forward 22.8 -> 22.0 us, step 0.1035-0.1039 ->
// 0.1027-0.1031 ms; fp32 unchanged within noise, so it keeps the default (tools/var_specs/ntst.py,
// profiles/r05nt; nt on every activation store made the fp32 forward 60 -> 66 us)
template <typename T> constexpr int kAct1Cpol = sizeof(T) == 2 ? 2 : 0;

template <typename T, class O = ObsDirect>
DEV void conv12_fwd_body(const uint8_t* __restrict__ x, const T* __restrict__ w1,
                         const float* __restrict__ b1, const T* __restrict__ w2,
                         const float* __restrict__ b2, T* __restrict__ act1,
                         uint32_t* __restrict__ mask, T* __restrict__ act2, int N, int fpw,
                         const C3Tail<T>& c3, int wg, T* __restrict__ smem, const O& rm = O{}) {
  using F = Frag<T>;
  typedef typename F::vec V;
  constexpr int KPL = F::KPL, KS = F::KSTEP;
  constexpr int LDI = c1::LF<T>::LDI;
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int LDA1 = OC1 + VEC;                    // act1 tile row (elements)
  constexpr int NKS1 = K1 / KS, NKS2 = K2 / KS;
  constexpr int G = c12f_groups<T>();
  // act1 tile rows: row y * A1P + x (y, x < 15).  The pitch of 22 rows per act1 row makes the
  // conv2 B fragment reads (16 output pixels x 16-byte chunks) conflict-free (tools/ldsbank.py
  // search_a1_pitch: 1.00x, against 1.67x for pitches 15 and 16)
  constexpr int A1P = 22;
  // (16 act1 rows: wave 3's pad tile oy = 15 writes row 15, read by nobody)
  constexpr int IMGSZ = c1::FROWS * LDI, GSZ = IMGSZ + A1P * 16 * LDA1;
  constexpr bool W2REG = sizeof(T) == 2;             // bf16: conv2 weights in registers
  // conv3 tail (bf16): the frames' act2 in LDS rows of LDA2 elements (144 B), 7 cells per
  // pixel row (a pad column): the conv3 window reads 2.0x instead of 3.0x, stores 2.0x
  // instead of 1.67x (tools/ldsbank.py)
  constexpr int LDA2 = OC2 + VEC, A2W = C12FLds<T>::A2W, A2F = H2 * A2W;
  constexpr int A2SZ = c3t_fmax<T>() * A2F * LDA2;
  static_assert(G * GSZ + A2SZ <= C12FLds<T>::ELEMS && GSZ == C12FLds<T>::GSZ, "LDS layout");
  T* a2s = smem + G * GSZ;
  const bool tail = c3.act3 != nullptr;
  constexpr int WPG = c12f_wpg<T>(), NTG = 64 * WPG;
  const int grp = (int)threadIdx.x / NTG, tid = (int)threadIdx.x % NTG, lane = tid & 63, wave = tid >> 6;
  const int wq = wave & 3, wh = WPG == 8 ? wave >> 2 : 0;
  constexpr int NI = WPG == 8 ? 1 : 2;  // conv1 output-channel tiles per wave
  // the image loads / stash run on 256 threads: fp32 on waves 4..7, during waves 0..3's conv2
  const bool ldr = WPG == 8 ? wh == 1 : tid < 256;
  const int ltid = WPG == 8 ? tid - 256 : tid;
  // the image is bf16 in both modes: the bytes 0..255 are exact in bf16.  fp32 runs conv1 as
  // three exact bf16 MFMA passes (W1 split hi + mid + lo, below) over it.
  using FB = Frag<__bf16>;
  typedef FB::vec VB;
  constexpr int ILDI = c1::LF<__bf16>::LDI, NKB1 = K1 / FB::KSTEP;
  static_assert(sizeof(T) == 4 || ILDI == LDI, "bf16 image layout");
  __bf16* img = reinterpret_cast<__bf16*>(smem + grp * GSZ);
  T* a1s = smem + grp * GSZ + IMGSZ;
  const int klb = FB::KPL * (lane >> 4);
  const int f0 = wg * fpw, f1 = min(N, f0 + fpw);
  const int kl = KPL * (lane >> 4);
  uint4 nv[3];
  if (ldr && f0 + grp < f1) c1_load_frame<T>(x + rm.map(f0 + grp) * IMG, ltid, nv);
  // biases: 16-byte loads issued with the frame, ahead of the weights (waiting for the weights
  // then covers them: loads retire in order)
  float bb1[2][4], bb2[4];
  // fp32: the conv2 bias of this lane's 4x4x1-block output channel (loaded in the frame loop, it
  // cost a wait for every load in flight there, the next frame's image included: 0.7-1.3k
  // clocks per frame, tools/var_specs/fwdstash32.py r04v4)
  const float bb2q = b2[16 * wq + 4 * ((lane >> 2) & 3) + (lane >> 4)];
  {
    const f32x4 u0 = *reinterpret_cast<const f32x4*>(b1 + 4 * (lane >> 4));
    const f32x4 u1 = *reinterpret_cast<const f32x4*>(b1 + 16 + 4 * (lane >> 4));
    const f32x4 u2 = *reinterpret_cast<const f32x4*>(b2 + 16 * wq + 4 * (lane >> 4));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bb1[0][q] = u0[q];
      bb1[1][q] = u1[q];
      bb2[q] = u2[q];
    }
  }
  // Weights: every wave needs all of W1 and its 16 rows of W2 as MFMA fragments.  For bf16
  // both are staged once per workgroup through LDS with coalesced 16-byte loads (76 KB per
  // workgroup instead of 8 waves x 28 KB of fragment loads through the CU's L2 port).
  // conv1 A fragments, rows oc = 16 i + (lane & 15), all of K: bf16 W1 (bf16 mode) or fp32 W1
  // split exactly into three bf16 terms x = hi + mid + lo (fp32 mode: round-to-nearest 8-bit
  // pieces of a 24-bit significand; each product with an image byte is exact in the fp32
  // accumulator, so the three passes give the fp32 products)
  VB wa1[NI][NKB1][sizeof(T) == 4 ? 3 : 1];
  const T* w2row = w2 + (size_t)(16 * wq + (lane & 15)) * K2 + kl;  // conv2: oc tile = wq
  // bf16: this wave's W2 rows in registers for the whole frame run (64 VGPRs).  fp32 reads its
  // fragments from L2 per k-step: holding all 128 VGPRs of them made the kernel 3.5 us slower
  // (78.9 -> 82.4 us, r03 q32 run)
  V wa2[W2REG ? NKS2 : 1];
  if constexpr (W2REG) {
    // rows padded by 16 (row step 8 mod 32 dwords): conflict-free b128 fragment reads.  The rows
    // sit in the act1 tiles (and past the act2 tiles), not over the images, so each group takes
    // its first frame into its image while the weights load
    constexpr int LW1 = K1 + 2 * VEC, LW2 = K2 + 2 * VEC, NT = 256 * G;
    constexpr int NV1 = OC1 * K1 / VEC, NV2 = OC2 * K2 / VEC;
    static_assert(G == 2 && OC1 * LW1 <= GSZ - IMGSZ && GSZ + IMGSZ + OC2 * LW2 <= C12FLds<T>::ELEMS,
                  "weight staging beside the images");
    T* w1s = smem + IMGSZ;
    T* w2s = smem + GSZ + IMGSZ;
    constexpr int NPT = (NV1 + NV2 + NT - 1) / NT;
    V wv[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = (int)threadIdx.x + i * NT;
      if (e < NV1) wv[i] = *reinterpret_cast<const V*>(w1 + (size_t)e * VEC);
      else if (e < NV1 + NV2) wv[i] = *reinterpret_cast<const V*>(w2 + (size_t)(e - NV1) * VEC);
    }
    // the frame was loaded first: waiting for it leaves the weight loads in flight
    if (ldr && f0 + grp < f1) c1_stash_frame_rot<__bf16, ILDI>(img, ltid, nv);
    if (ldr && f0 + grp + G < f1) c1_load_frame<T>(x + rm.map(f0 + grp + G) * IMG, ltid, nv);
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = (int)threadIdx.x + i * NT;
      if (e < NV1) {
        *reinterpret_cast<V*>(w1s + (e / (K1 / VEC)) * LW1 + (e % (K1 / VEC)) * VEC) = wv[i];
      } else if (e < NV1 + NV2) {
        const int e2 = e - NV1;
        *reinterpret_cast<V*>(w2s + (e2 / (K2 / VEC)) * LW2 + (e2 % (K2 / VEC)) * VEC) = wv[i];
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int ks = 0; ks < NKS1; ++ks)
        wa1[i][ks][0] = *reinterpret_cast<const V*>(w1s + (16 * i + (lane & 15)) * LW1 + ks * KS + kl);
#pragma unroll
    for (int ks = 0; ks < NKS2; ++ks)
      wa2[ks] = *reinterpret_cast<const V*>(w2s + (16 * wave + (lane & 15)) * LW2 + ks * KS + kl);
    __syncthreads();  // the staging area becomes the frame tiles
  } else {
    // fp32: W1 staged once as its three bf16 planes (c1_stage_w1_f32, the split of c1_load_w1),
    // the fragments read from LDS
    static_assert(3 * OC1 * C1W_LD * 2 <= (int)sizeof(T) * G * GSZ, "W1 plane staging");
    __bf16* w1p = reinterpret_cast<__bf16*>(smem);
    if (threadIdx.x < 256) c1_stage_w1_f32(reinterpret_cast<const float*>(w1), w1p, (int)threadIdx.x);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int kb = 0; kb < NKB1; ++kb)
#pragma unroll
        for (int tm = 0; tm < 3; ++tm)
          wa1[i][kb][tm] = *reinterpret_cast<const VB*>(
              w1p + (tm * OC1 + 16 * (NI == 1 ? wh : i) + (lane & 15)) * C1W_LD + kb * FB::KSTEP + klb);
    __syncthreads();  // the staging area becomes the frame tiles
  }
  // consume the bias loads here: waits for them placed inside the loop would (merged over the
  // back-edge) also stall every iteration on its in-flight frame prefetch
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    asm volatile("" ::"v"(bb1[0][q]), "v"(bb1[1][q]), "v"(bb2[q]));
  }
  asm volatile("" ::"v"(bb2q));
  const int n_it = (f1 - f0 + G - 1) / G;
  // conv1 pixel tiles of this wave: rows oy = wave, wave + 4, wave + 8, wave + 12 of the 15x15
  // output (lane & 15 = ox; ox = 15 and wave 3's oy = 15 are pad lanes / a pad tile).  The tiles
  // run in two pairs: the second pair's MFMAs are issued while the first pair's epilogue
  // (scale, bias, ReLU, bf16 pack, mask bits, stores) runs on the VALU.
  int c1base[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) c1base[t] = (min(wq + 4 * t, 14) * c1::GRID + (lane & 15)) * ILDI;
  auto c1_off = [&](int kb) {  // bf16 fragment k-block kb: this lane's 8 k = 8 channels of one tap
    const int k = kb * FB::KSTEP + klb, tap = k / c1::CH, ch = k - tap * c1::CH;
    return ((tap >> 1) * c1::GRID + (tap & 1)) * ILDI + ch;
  };
  // conv2: 3 pixel tiles (3 accumulators), B fragments one k-step ahead
  // fp32: pixel tile 2 holds only pixels 32..35; they run on 4x4x1 blocks (see the conv2 loop),
  // whose B operand is pixel 32 + (lane & 3) at k-phase lane >> 4
  int c2row[3];
#pragma unroll
  for (int pt = 0; pt < 3; ++pt) {
    const int px = (pt == 2 && !W2REG) ? 32 + (lane & 3) : min(pt * 16 + (lane & 15), P2 - 1);
    const int oy = px / H2, ox = px - oy * H2;
    c2row[pt] = ((ST2 * oy) * A1P + ST2 * ox) * LDA1 + kl;
  }
  auto c2_off = [&](int ks) {
    const int k = ks * KS, tap = k >> 5, ci = k & 31;
    return ((tap >> 2) * A1P + (tap & 3)) * LDA1 + ci;
  };
  // Branch-free epilogue stores: act1 and the mask go through buffer stores whose pad lanes
  // carry an out-of-range offset (dropped by the hardware bounds check); pad lanes' LDS act1
  // stores land in the tile's unused pitch columns / pad rows.
  const __amdgpu_buffer_rsrc_t rs_act1 =
      __builtin_amdgcn_make_buffer_rsrc(act1, 0, N * c1::NPIX * OC1 * (int)sizeof(T), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_mask =
      __builtin_amdgcn_make_buffer_rsrc(mask, 0, N * c1::NPIX * 4, 0x00020000);
  constexpr int OOB = 0x7ffffff0;
  auto c1_mma = [&](f32x4 (&acc)[2][NI], int t0) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ii = 0; ii < NI; ++ii) acc[u][ii] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int NT = sizeof(T) == 4 ? 3 : 1;  // W1 terms
    VB bq[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u) bq[0][u] = *reinterpret_cast<const VB*>(img + c1base[t0 + u] + c1_off(0));
#pragma unroll
    for (int kb = 0; kb < NKB1; ++kb) {
      if (kb + 1 < NKB1) {
        const int off = c1_off(kb + 1);
#pragma unroll
        for (int u = 0; u < 2; ++u) bq[(kb + 1) & 1][u] = *reinterpret_cast<const VB*>(img + c1base[t0 + u] + off);
      }
#pragma unroll
      for (int tm = 0; tm < NT; ++tm)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int ii = 0; ii < NI; ++ii) acc[u][ii] = FB::mma(wa1[ii][kb][tm], bq[kb & 1][u], acc[u][ii]);
    }
  };
  auto c1_epi = [&](const f32x4 (&acc)[2][NI], int t0, int f) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int oy = wq + 4 * (t0 + u), ox = lane & 15;
      const bool st = oy < H1 && ox < H1;
      const int pc = oy * H1 + ox;               // act1 / mask pixel (15 x 15)
      T* arow = a1s + (oy * A1P + ox) * LDA1;    // LDS act1 row (pad lanes: unused slots)
      const int gofs = st ? (int)((((size_t)f * c1::NPIX + pc) * OC1) * sizeof(T)) : OOB;
      uint32_t bits = 0;
#pragma unroll
      for (int ii = 0; ii < NI; ++ii) {
        const int i = NI == 1 ? wh : ii;  // output-channel tile
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float xv = acc[u][ii][q] * (1.f / 255.f) + bb1[i][q];
          v[q] = fmaxf(xv, 0.f);
          // ReLU mask bit = (x > 0): the float's bits as a signed int are > 0 exactly then
          // (one v_med3_i32)
          bits |= (uint32_t)min(max((int)__float_as_uint(xv), 0), 1) << (16 * i + 4 * (lane >> 4) + q);
        }
        const int oc = 16 * i + 4 * (lane >> 4);
        store4(arow + oc, v);
        if constexpr (sizeof(T) == 2) {
          const i32x2 d = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
          __builtin_amdgcn_raw_buffer_store_b64(d, rs_act1, gofs + oc * 2, 0, kAct1Cpol<T>);
        } else {
          const i32x4 d = {(int)__float_as_uint(v[0]), (int)__float_as_uint(v[1]),
                           (int)__float_as_uint(v[2]), (int)__float_as_uint(v[3])};
          __builtin_amdgcn_raw_buffer_store_b128(d, rs_act1, gofs + oc * 4, 0, kAct1Cpol<T>);
        }
      }
      bits = xor32_or(xor16_or(bits));
      if constexpr (NI == 2) {
        __builtin_amdgcn_raw_buffer_store_b32((int)bits, rs_mask,
                                              st && lane < 16 ? (int)(((size_t)f * c1::NPIX + pc) * 4) : OOB,
                                              0, 0);
      } else {  // this wave's 16 bits (oc tile wh) into its half of the pixel's mask word
        __builtin_amdgcn_raw_buffer_store_b16((short)(bits >> (16 * wh)), rs_mask,
                                              st && lane < 16 ? (int)(((size_t)f * c1::NPIX + pc) * 4 + 2 * wh) : OOB,
                                              0, 0);
      }
    }
  };
  // fp32: the group's first frame goes into the image now (the weight staging area is free), and
  // the second is fetched (bf16 did both during its weight staging); every later frame is staged
  // during the previous frame's conv2
  if constexpr (!W2REG) {
    if (ldr && f0 + grp < f1) c1_stash_frame_rot<__bf16, ILDI>(img, ltid, nv);
    if (ldr && f0 + grp + G < f1) c1_load_frame<T>(x + rm.map(f0 + grp + G) * IMG, ltid, nv);
    __syncthreads();
  }
  for (int it = 0; it < n_it; ++it) {
    const int f = f0 + G * it + grp;
    const bool active = f < f1;
    V ar0[3];  // fp32: conv2's first W2 fragments, loaded under this frame's conv1
    if (active) {
      // ---- conv1 -> act1 (HBM + LDS) and its ReLU bit mask ----
      f32x4 accA[2][NI], accB[2][NI];
      // issued here, 4.6k clocks ahead of their use: loaded at the top of the conv2 loop, the
      // first MFMA of every frame waited a whole L2 round trip (forward 60.2 -> 58.8 us,
      // tools/var_specs/w2early.py r04v7)
      if constexpr (!W2REG) {
#pragma unroll
        for (int d = 0; d < 3; ++d) ar0[d] = F::load(w2row + d * KS);
      }
      c1_mma(accA, 0);
      c1_mma(accB, 2);
      c1_epi(accA, 0, f);
      c1_epi(accB, 2, f);
    }
    __syncthreads();  // the act1 tile is complete; the image is free
    if (active) {
      // ---- conv2 from the LDS act1 tile -> act2, and the next frame into the image ----
      f32x4 acc[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                      f32x4{0.f, 0.f, 0.f, 0.f}};
      V bq[2][3];
      constexpr int NPT = W2REG ? 3 : 2;  // 16-pixel tiles in slots 0 .. NPT-1
      const bool c2w = WPG == 4 || wh == 0;  // fp32: conv2 on waves 0..3, the stash on 4..7
      if (c2w) {
#pragma unroll
      for (int pt = 0; pt < 3; ++pt)
        if (pt < NPT || pt == 2) bq[0][pt] = *reinterpret_cast<const V*>(a1s + c2row[pt] + c2_off(0));
      // fp32: the W2 fragments stream from L2 in a ring PD2 k-steps ahead of their MFMAs (the
      // order pinned by scheduling barriers; the compiler kept them one step ahead)
      constexpr int PD2 = W2REG ? 1 : 4;
      static_assert(W2REG || PD2 - 1 == 3, "ar0 holds the ring's first PD2 - 1 fragments");
      V ar[PD2];
      if constexpr (!W2REG) {
#pragma unroll
        for (int d = 0; d < PD2 - 1; ++d) ar[d] = ar0[d];
      }
#pragma unroll
      for (int ks = 0; ks < NKS2; ++ks) {
        if constexpr (!W2REG) {
          if (ks + PD2 - 1 < NKS2) ar[(ks + PD2 - 1) % PD2] = F::load(w2row + (ks + PD2 - 1) * KS);
        }
        if (ks + 1 < NKS2) {
          const int off = c2_off(ks + 1);
#pragma unroll
          for (int pt = 0; pt < 3; ++pt)
            if (pt < NPT || pt == 2) bq[(ks + 1) & 1][pt] = *reinterpret_cast<const V*>(a1s + c2row[pt] + off);
        }
        V a;
        if constexpr (W2REG) a = wa2[ks];
        else a = ar[ks % PD2];
        if constexpr (!W2REG) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < F::NE; ++e) {
          if constexpr (W2REG) {
#pragma unroll
            for (int pt = 0; pt < 3; ++pt) acc[pt] = F::mma_e(e, a, bq[ks & 1][pt], acc[pt]);
          } else {
            // pixels 0..31: two 16x16x4 tiles; 32..35: one v_mfma_f32_4x4x1_16b_f32 (block
            // 4 g + og = oc rows 4 og .. 4 og + 3 of the same W2 element, k-phase g, pixel
            // 32 + j) instead of a quarter-full third tile
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) acc[pt] = F::mma_e(e, a, bq[ks & 1][pt], acc[pt]);
            acc[2] = __builtin_amdgcn_mfma_f32_4x4x1f32(a[e], bq[ks & 1][2][e], acc[2], 0, 0, 0);
          }
        }
        if constexpr (!W2REG) __builtin_amdgcn_sched_barrier(0);
      }
      }
      if (ldr && f + G < f1) c1_stash_frame_rot<__bf16, ILDI>(img, ltid, nv);
      if (ldr && f + 2 * G < f1) c1_load_frame<T>(x + rm.map(f + 2 * G) * IMG, ltid, nv);
      if (!W2REG && wh == 0) {
        // the 4x4x1 blocks: lane 16 g + 4 og + j holds act2[pixel 32 + j][oc 16 w + 4 og + reg]
        // over k-phase g; ((g0 + g1) + (g2 + g3)) of reg q lands on row q (rows_sum4), so lane
        // 16 q + 4 og + j stores one value
        const int pc = 32 + (lane & 3), oc = 16 * wq + 4 * ((lane >> 2) & 3) + (lane >> 4);
        const float v = fmaxf(rows_sum4(acc[2][0], acc[2][1], acc[2][2], acc[2][3]) + bb2q, 0.f);
        act2[((size_t)f * P2 + pc) * OC2 + oc] = (T)v;
        if (tail) {
          const int cy = pc / H2, cx = pc - cy * H2;
          a2s[((f - f0) * A2F + cy * A2W + cx) * LDA2 + oc] = (T)v;
        }
      }
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) {
        const int pc = pt * 16 + (lane & 15);
        if (c2w && pc < P2) {
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = fmaxf(acc[pt][q] + bb2[q], 0.f);
          store4(act2 + ((size_t)f * P2 + pc) * OC2 + 16 * wq + 4 * (lane >> 4), v);
          if (tail) {
            const int cy = pc / H2, cx = pc - cy * H2;
            store4(a2s + ((f - f0) * A2F + cy * A2W + cx) * LDA2 + 16 * wq + 4 * (lane >> 4), v);
          }
        }
      }
    }
    __syncthreads();  // the image holds the next frame; the act1 tile is free
  }
  if constexpr (W2REG) {
    if (tail) {
      // ---- conv3 + ReLU + LayerNorm of this workgroup's frames (the frame loop ended with a
      // barrier: the image / act1 areas are free, act2 is in a2s) ----
      // W3 rows of 592 (row step 8 mod 64 dwords: the k-contiguous b128 reads are conflict-free
      // by tools/ldsbank.py; 584 is 2.0x)
      constexpr int LDW3 = K3 + 2 * VEC, LDE = OC3 + 4, NT = 256 * G;
      constexpr int NV3 = OC3 * K3 / VEC, NPT3 = (NV3 + NT - 1) / NT;
      static_assert(OC3 * LDW3 + C3T_FMAX * P3 * LDE * 2 <= G * GSZ, "conv3 tail LDS");
      static_assert(C3T_FMAX <= 4 * G, "one wave per frame");
      T* w3s = smem;
      float* ets = reinterpret_cast<float*>(smem + OC3 * LDW3);
      V wv3[NPT3];
#pragma unroll
      for (int i = 0; i < NPT3; ++i) {
        const int e = min((int)threadIdx.x + i * NT, NV3 - 1);
        wv3[i] = *reinterpret_cast<const V*>(c3.w3 + (size_t)e * VEC);
      }
      const int gw = (int)threadIdx.x >> 6, nF = f1 - f0;
      const LnLane lk = ln_lane_consts(lane, c3.b3, c3.gam, c3.bet);
#pragma unroll
      for (int i = 0; i < NPT3; ++i) {
        const int e = (int)threadIdx.x + i * NT;
        if (e < NV3) *reinterpret_cast<V*>(w3s + (e / (K3 / VEC)) * LDW3 + (e % (K3 / VEC)) * VEC) = wv3[i];
      }
      __syncthreads();
      if (gw < nF) {
        const int p = lane & 15, oy = p >> 2, ox = p & 3;
        const T* a2f = a2s + (gw * A2F + oy * A2W + ox) * LDA2 + kl;
        f32x4 acc3[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                         f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int ks = 0; ks < K3 / KS; ++ks) {  // k = ks*32 + kl: tap = k / 64, ci = k % 64
          const int k = ks * KS, tap = k >> 6, kh = tap / 3, kw = tap - kh * 3;
          const V b = *reinterpret_cast<const V*>(a2f + (kh * A2W + kw) * LDA2 + (k & 63));
          V a[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const V*>(w3s + (16 * i + (lane & 15)) * LDW3 + k + kl);
#pragma unroll
          for (int e = 0; e < F::NE; ++e)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc3[i] = F::mma_e(e, a[i], b, acc3[i]);
        }
        float* et = ets + gw * P3 * LDE;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          *reinterpret_cast<f32x4*>(et + p * LDE + 16 * i + 4 * (lane >> 4)) = acc3[i];
        if (c3.y_sc1)
          ln_frame_epilogue<T, true>(et, LDE, f0 + gw, lane, lk, c3.act3, c3.y, c3.stats);
        else
          ln_frame_epilogue<T>(et, LDE, f0 + gw, lane, lk, c3.act3, c3.y, c3.stats);
      }
    }
  }
  if constexpr (!W2REG) {
    if (tail) {
      // ---- fp32 conv3 + ReLU + LayerNorm of this workgroup's frames (the frame loop ended
      // with a barrier: the image / act1 areas are free, act2 is in a2s).  Wave w computes oc
      // tile w of every frame: its W3 rows (the A operand, 144 VGPRs) by 16-byte loads, the act2
      // window of each output pixel from LDS; the same k-step order and fragments as
      // gemm_tile<Conv3LnFwd> and the same ln_frame_epilogue, so act3 / y / stats are
      // bit-identical to the separate conv3 launch. ----
      constexpr int FMAX = c3t_fmax<T>(), NKS3 = K3 / KS, LDE = OC3 + 4;
      static_assert(FMAX * P3 * LDE <= G * GSZ, "fp32 conv3 tail LDS");
      // The 36 fragment loads are issued PD3 k-steps ahead of the MFMAs that use them, inside
      // the k-loop: issued all at once, the burst of every CU's 147 KB of W3 stalls the load
      // issue itself (per-CU load bandwidth, ~17 B/clk) for ~7k cycles before the first MFMA
      // (r03 stamps)
      constexpr int PD3 = 8;
      const int nF = f1 - f0;
      const LnLane lk = ln_lane_consts(lane, c3.b3, c3.gam, c3.bet);
      float* ets = reinterpret_cast<float*>(smem);
      if (wh == 0) {  // (8 waves: the first four run the conv3 GEMM, all eight the LayerNorm)
        V w3a[NKS3];
        const T* w3row = c3.w3 + (size_t)(16 * wq + (lane & 15)) * K3 + kl;
#pragma unroll
        for (int ks = 0; ks < PD3; ++ks) w3a[ks] = F::load(w3row + ks * KS);
        const int p = lane & 15, oy = p >> 2, ox = p & 3;
        const T* a2f = a2s + (oy * A2W + ox) * LDA2 + kl;
        f32x4 acc3[FMAX];
#pragma unroll
        for (int fr = 0; fr < FMAX; ++fr) acc3[fr] = f32x4{0.f, 0.f, 0.f, 0.f};
        // every frame slot runs (a slot past the run re-reads the last frame; its result is
        // dropped), so the FMAX accumulators interleave (F::mma_e); the act2 window reads run one
        // k-step ahead (k = ks*16 + kl: tap = k / 64, ci = k % 64)
        auto bload = [&](int ks, V* b) {
          const int k = ks * KS, tap = k >> 6, kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
          for (int fr = 0; fr < FMAX; ++fr)
            b[fr] = *reinterpret_cast<const V*>(a2f + (min(fr, nF - 1) * A2F + kh * A2W + kw) * LDA2 + (k & 63));
        };
        V b[2][FMAX];
        bload(0, b[0]);
#pragma unroll
        for (int ks = 0; ks < NKS3; ++ks) {
          if (ks + PD3 < NKS3) w3a[ks + PD3] = F::load(w3row + (ks + PD3) * KS);
          if (ks + 1 < NKS3) bload(ks + 1, b[(ks + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int e = 0; e < F::NE; ++e)
#pragma unroll
            for (int fr = 0; fr < FMAX; ++fr) acc3[fr] = F::mma_e(e, w3a[ks], b[ks & 1][fr], acc3[fr]);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int fr = 0; fr < FMAX; ++fr)
          if (fr < nF) *reinterpret_cast<f32x4*>(ets + (fr * P3 + p) * LDE + 16 * wq + 4 * (lane >> 4)) = acc3[fr];
      }
      __syncthreads();
      if constexpr (WPG == 8) {  // one frame per wave
        static_assert(FMAX <= 8, "a wave per frame");
        if (wave < nF) {
          const int fr1[1] = {f0 + wave};
          ln_frames_epilogue<T, 1>(ets + wave * P3 * LDE, 0, LDE, fr1, lane, lk, c3.act3, c3.y, c3.stats);
        }
      } else {
        // frames wave and wave + 4 (FMAX <= 8) in one interleaved pass
        static_assert(FMAX <= 8, "two frames per wave");
        if (wave + 4 < nF) {
          const int fr2[2] = {f0 + wave, f0 + wave + 4};
          ln_frames_epilogue<T, 2>(ets + wave * P3 * LDE, 4 * P3 * LDE, LDE, fr2, lane, lk, c3.act3, c3.y, c3.stats);
        } else if (wave < nF) {
          const int fr1[1] = {f0 + wave};
          ln_frames_epilogue<T, 1>(ets + wave * P3 * LDE, 0, LDE, fr1, lane, lk, c3.act3, c3.y, c3.stats);
        }
      }
    }
  }
}

template <typename T, class O = ObsDirect>
__global__ __launch_bounds__(c12f_threads<T>()) void conv12_fwd_s2d(
    const uint8_t* __restrict__ x, const T* __restrict__ w1, const float* __restrict__ b1,
    const T* __restrict__ w2, const float* __restrict__ b2, T* __restrict__ act1,
    uint32_t* __restrict__ mask, T* __restrict__ act2, int N, int fpw, const C3Tail<T> c3,
    unsigned long long* __restrict__ step_stamp, const O rm) {
  __shared__ __attribute__((aligned(16))) T smem[C12FLds<T>::ELEMS];
  // the device step clock (impala_step_clock): the learner step's first kernel stamps the
  // constant 100 MHz clock as its first workgroup starts (one vector store; nullptr = off)
  if (step_stamp != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
    *step_stamp = __builtin_amdgcn_s_memrealtime();
  conv12_fwd_body<T, O>(x, w1, b1, w2, b2, act1, mask, act2, N, fpw, c3, (int)blockIdx.x, smem, rm);
}

// ---------------------------------------------------------------------------------------
// conv2 input gradient + ReLU mask + conv1 weight gradient, one frame at a time, fused:
//
//   dY1[p][ci] = [act1 > 0] * sum_{kh,kw,oc: iy = 2 oy + kh, ix = 2 ox + kw} dY2[oy][ox][oc] W2[oc][kh][kw][ci]
//   dW1'[oc][k'] += sum_p dY1[p][oc] * s2d[row(p, tap)][ch]     (1/255 at the end)
//
// dY1 (the 15x15x32 conv2 input gradient) never leaves LDS.  The conv2 dgrad is split into the
// four stride-parity classes (iy % 2, ix % 2): each class is a GEMM [32 ci] x [8x8 cells] with
// K = 4 taps x 64 oc, and wave w owns class w for the whole kernel, so its W2 fragments (the
// A operand, ci x oc) stay in registers; the B operand is a 16-byte LDS read of the frame's
// dY2 held in a zero-bordered 9x9 cell grid (no bounds tests).  The ReLU mask of act1 comes
// from the bit mask conv1_fwd_s2d writes (one 32-bit word per pixel).  The conv1 weight
// gradient then reads dY1 and the frame's s2d image from LDS: wave w owns tap w (48 channels
// = 3 column tiles) for both 16-row oc tiles.  Each workgroup takes a contiguous run of frames
// and writes one fp32 partial slab [32][192] (k' order) + bias sums, reduced by reduce_grads.
// ---------------------------------------------------------------------------------------
// lane move within rows of 16 lanes (DPP row_shr / row_shl); lanes without a source get 0
template <int CTRL, typename V>
DEV V dpp_move(const V& v) {
  constexpr int NW = sizeof(V) / 4;
  union U { V v; int w[NW]; } a, r;
  a.v = v;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = __builtin_amdgcn_update_dpp(0, a.w[i], CTRL, 0xF, 0xF, false);
  return r.v;
}
template <typename V>
DEV V vor(const V& x, const V& y) {  // bitwise OR (one side is all-zero bits lane-wise)
  constexpr int NW = sizeof(V) / 4;
  union U { V v; int w[NW]; } a, b, r;
  a.v = x;
  b.v = y;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = a.w[i] | b.w[i];
  return r.v;
}

namespace c12 {
constexpr int QG = 9;                          // dY2 cell grid: oy = r - 1, r in [0, 9)
constexpr int NCELL = QG * QG;
}  // namespace c12

// G 4-wave groups per workgroup take alternating frames of the run (G frames in flight per CU
// on top of the one-frame register prefetch); their partials are summed in a fixed order.
// (fp32: two 4-wave groups with different roles, see conv12_bwd_body_f32)
template <typename T> constexpr int c12_groups() { return 2; }

// fp32 body (conv12_bwd_body_f32) LDS, in 4-byte words, double-buffered per frame where the
// two groups overlap: the frame's s2d image as BYTES (the raw 0..255 values, converted when
// read) in [Y][channel][X] rows of XP bytes (4 consecutive X in one 32-bit word) x 2, dY1 in
// pixel rows iy * 16 + ix (240: the conv1 weight gradient's 15 k-steps = the 15 pixel rows,
// ix = 15 a zero pad) x 2, dY2 rows (36) x 2, one half-Z tile per stride-parity class (2 taps x 32 channels; row 36
// stays zero: the gather's out-of-range taps read it), the mask words x 2.
// The Z rows are 64 floats = 16 chunks of 16 B, unpadded; chunk c of row r is stored at chunk
// c ^ zswz(r) (ZSWZ).  The Z stores write 8 consecutive rows at one chunk per ds_write_b128 lane
// group (bank = address mod 128 B: zswz(r) mod 8 is a permutation of r mod 8), and a gather
// read's 16-lane group (ds_read_b128 groups, MI355X_MICROARCH.md §LDS) takes chunks 0..3 of row r,
// 4..7 of rows r + 1 and r + 2, 0..3 of row r + 3 (+ 8 per tap j2), for any r: bit 3 and bit 2
// of zswz follow the row's parity, so the four 64-byte pieces land in four different quarters of
// the 256-byte bank row.  With the round-3 pitch (68 floats) the same reads overlapped by up to
// 3 chunks (39 % of the backward's LDS cycles were conflict cycles, profiles/r04pmc).
struct C12B32 {
  static constexpr bool ZSWZ = true;
  // group B's conv1 weight gradient split over k (WKS): wave w takes k-blocks 2 w, 2 w + 1 of
  // all four taps (the dY1 split into bf16 terms done once per value, not once per tap), the
  // partials summed in wave order at the end; else wave w takes tap w over all eight k-blocks
  static constexpr bool WKS = true;
  static constexpr int XP = 20, LDX = c1::LB<float>::LDX;  // image row bytes (X 0..16), dY1 row
  static constexpr int NROW = 240, LDD = OC2 + 4, DROWS = P2, LDZ = 2 * OC1 + (ZSWZ ? 0 : 4),
                       ZROWS = P2 + 1;
  static_assert(2 * OC1 == 64, "Z rows of 16 chunks");
  __device__ static constexpr int zswz(int r) { return ZSWZ ? ((r & 1) * 12) | ((r >> 1) & 3) : 0; }
  static constexpr int IMGW = c1::GRID * c1::CH * XP / 4, DYW = NROW * LDX, D2W = DROWS * LDD;
  static constexpr int IMG = 0, DYT = IMG + 2 * IMGW, D2S = DYT + 2 * DYW;
  static constexpr int Z0 = D2S + 2 * D2W, ZSZ = ZROWS * LDZ, MSK = Z0 + 4 * ZSZ;
  static constexpr int BYTES = (MSK + 2 * c1::NPIX) * 4;
};

// LDS of the body (bytes): per-group image / dY1 / dY2 tiles, the ReLU mask words, bias sums
template <typename T> struct C12BLds {
  static constexpr int VEC = 16 / (int)sizeof(T), LDX = c1::LB<T>::LDX, LD2 = c1::LB<T>::LD2;
  static constexpr int IMGSZ = c1::GRID * c1::GRID * c1::LB<T>::LDI, DYSZ = c1::NPAD * LDX;
  static constexpr int G = c12_groups<T>();
  static constexpr int GSZ = IMGSZ + DYSZ + c12::NCELL * LD2;
  static constexpr int MSK = (G * GSZ * (int)sizeof(T) + 15) / 16 * 16;
  static constexpr int BRED = MSK + (G * c1::NPIX * 4 + 15) / 16 * 16;
  static constexpr int BYTES = sizeof(T) == 4 ? C12B32::BYTES : BRED + 4 * G * OC1 * 4;
};

// The W2 fragments of stride-parity class `cls` (conv12_bwd_body_f32's group A wave):
// B[k = oc][n = ci] = W2[oc][kh][kw][ci] for the class's 4 taps, 16-byte loads from the
// transposed copy w2t[(kh*4+kw)*32 + ci][oc] (k = oc contiguous)
DEV void c12_load_w2(const float* __restrict__ w2t, Frag<float>::vec (&wb)[4][OC2 / Frag<float>::KSTEP][2],
                     int cls, int lane, int t0 = 0, int t1 = 4) {  // taps [t0, t1)
  using F = Frag<float>;
  constexpr int KS = F::KSTEP, NKO = OC2 / KS;
  // 32-bit element offsets from the (uniform) base, from a lane value the compiler cannot hoist:
  // a caller inside a frame loop would otherwise keep 32 64-bit addresses live across it
  int ln = lane;
  asm volatile("" : "+v"(ln));
  const int py = cls >> 1, px = cls & 1;
  const uint32_t o0 = (uint32_t)((ln & 15) * OC2 + 4 * (ln >> 4));
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t < t0 || t >= t1) continue;
    const int kh = py + 2 * (t >> 1), kw = px + 2 * (t & 1);
#pragma unroll
    for (int ks = 0; ks < NKO; ++ks)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
        wb[t][ks][ct] = F::load(w2t + (o0 + (uint32_t)(((kh * KS2 + kw) * OC1 + 16 * ct) * OC2 + ks * KS)));
  }
}

// ---------------------------------------------------------------------------------------
// fp32 conv2 input gradient + ReLU mask + conv1 weight gradient, per frame, in SCATTER form:
//
//   Z[op][t][ci] = sum_oc dY2[op][oc] W2[oc][t][ci]        (36 conv2 output pixels op)
//   dY1[iy][ix][ci] = [act1 > 0] * sum_{t = (kh, kw): iy = 2 oy + kh, ix = 2 ox + kw} Z[op][t][ci]
//   dW1'[oc][k'] += sum_p dY1[p][oc] * s2d[row(p, tap)][ch]     (1/255 at the end)
//
// The 16 taps fall into the four stride-parity classes (kh % 2, kw % 2) and a class's 4 taps
// reach exactly the input pixels of that parity.  512 threads in two 4-wave groups with
// different roles, software-pipelined over the workgroup's frames (one barrier per step):
//   group A (waves 0..3), frame i:   wave w owns class w: Z for its 4 taps in two halves of 2
//       taps (rows op: 2 tiles of 16 + the last 4 on 4x4x1 blocks, cols (tap, ci), K = 64 oc;
//       its W2 fragments in registers), each half gathered into dY1[i & 1] in a fixed tap
//       order (the second half adds to the first half's partial sums, masks and keeps the
//       conv1 bias partials); then it stages frame i + 1's dY2 / mask (and frame i + 2's loads);
//   group B (waves 4..7), frame i - 1: the conv1 weight gradient, wave w owns tap w (48
//       channels = 3 column tiles) for both 16-row oc tiles, over dY1[(i - 1) & 1] and the
//       image bytes of frame i - 1.
// With one wave of each group per SIMD, the gather / staging work of one group runs under the
// other group's MFMAs (the one-group body ran every phase behind a workgroup barrier with one
// wave per SIMD).  Every value is the same fp32 sum in the same order as that body: the tap
// sums ((z0 + z1) + z2) + z3, oc in MFMA order, pixels in k-step order.  Each workgroup writes
// one fp32 partial slab [32][192] (k' order) + bias sums, reduced by reduce_grads.
// ---------------------------------------------------------------------------------------
template <int ROLE, class O = ObsDirect>
DEV void conv12_bwd_body_f32(const uint8_t* __restrict__ x, const float* __restrict__ w2t,
                             const float* __restrict__ dy2, const uint32_t* __restrict__ mask1,
                             float* __restrict__ slab, float* __restrict__ slab_bias, int N,
                             int fpw, int wg, char* __restrict__ lds,
                             Frag<float>::vec (&wb)[4][OC2 / Frag<float>::KSTEP][2], bool load_w2,
                             const O& rm = O{}) {
  using F = Frag<float>;
  typedef F::vec V;
  using L = C12B32;
  constexpr int KS = F::KSTEP, XP = L::XP, LDX = L::LDX, LDD = L::LDD, LDZ = L::LDZ;
  static_assert(L::NROW == H1 * 16 && H1 < 16 && c1::GRID == 16, "dY1 rows: 16 pixels per image row");
  constexpr int NKO = OC2 / KS;             // 4 k-steps over oc
  constexpr int D2V = P2 * OC2 / 4;         // float4 vectors of one dY2 frame (576)
  constexpr int ND2 = (D2V + 255) / 256;
  float* smem = reinterpret_cast<float*>(lds);
  // ROLE 0 / 1: this wave's group is known at compile time (the fused kernel runs each group as
  // its own code path); -1: decided per wave here
  const bool is_a = ROLE == 0 ? true : ROLE == 1 ? false : ((int)threadIdx.x >> 8) == 0;
  const int tid = (int)threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  const int f0 = wg * fpw, f1 = min(N, f0 + fpw), nF = max(f1 - f0, 0);
  const int kl = 4 * (lane >> 4);
  auto img_buf = [&](int b) { return reinterpret_cast<uint8_t*>(smem + L::IMG + b * L::IMGW); };
  auto dyt_buf = [&](int b) { return smem + L::DYT + b * L::DYW; };
  auto d2s_buf = [&](int b) { return smem + L::D2S + b * L::D2W; };
  auto msk_buf = [&](int b) { return reinterpret_cast<uint32_t*>(smem + L::MSK + b * c1::NPIX); };
  // ---- group A state ----
  const int py = wave >> 1, px = wave & 1;  // A: this wave's stride-parity class
  float* zw = smem + L::Z0 + wave * L::ZSZ;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};    // A: conv1 bias partials of this lane's 4 channels
  // A: W2 fragments wb[tap j1*2+j2][k-step][ci tile] (c12_load_w2; loaded here if load_w2)
  // ---- group B state ----
  // B: conv1 weight gradient [tap (WKS) ][oc tile i][ch tile j]
  constexpr int NTB = L::WKS ? 4 : 1;
  f32x4 acc[NTB][2][3];
#pragma unroll
  for (int t = 0; t < NTB; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // group B's staging, global loads then LDS stores (the latency runs under group A's work):
  // frame fi's image bytes -> IMG[bi] as [Y][channel c = ci * 16 + bb * 4 + d][X] bytes (a
  // 4 x 4 byte transpose of the 16 bytes a thread loads: 4 cells X x 4 columns d), frame fd's
  // dY2 rows / mask words -> D2S[bd] / MSK[bd]
  auto stage = [&](int fi, int bi, int fd, int bd) {
    uint4 nv[3];
    f32x4 nd2[ND2];
    uint32_t nmk = 0;
    if (fi >= 0) c1_load_frame<float>(x + rm.map(fi) * IMG, tid, nv);
    if (fd >= 0) {
      const float* src = dy2 + (size_t)fd * P2 * OC2;
#pragma unroll
      for (int i = 0; i < ND2; ++i) {
        const int e = tid + i * 256;
        nd2[i] = e < D2V ? *reinterpret_cast<const f32x4*>(src + e * 4) : F::zero();
      }
      if (tid < c1::NPIX) nmk = mask1[(size_t)fd * c1::NPIX + tid];
      float* d2s = d2s_buf(bd);
#pragma unroll
      for (int i = 0; i < ND2; ++i) {
        const int e = tid + i * 256;
        if (e < D2V) *reinterpret_cast<f32x4*>(d2s + ((e * 4) / OC2) * LDD + (e * 4) % OC2) = nd2[i];
      }
      if (tid < c1::NPIX) msk_buf(bd)[tid] = nmk;
    }
    if (fi < 0) return;
    uint8_t* img = img_buf(bi);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int vi = tid + i * 256, ci = vi >> 8, yy = (vi & 255) >> 2, xq = vi & 3;
      const int Y = yy >> 2, bb = yy & 3;
      const uint32_t w[4] = {nv[i].x, nv[i].y, nv[i].z, nv[i].w};  // word q: cell X = 4 xq + q
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint32_t t = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) t |= ((w[q] >> (8 * d)) & 255u) << (8 * q);
        *reinterpret_cast<uint32_t*>(img + (Y * c1::CH + ci * 16 + bb * 4 + d) * XP + 4 * xq) = t;
      }
    }
  };
  // group B's staging split in two for its loop: the loads issued at the top of a step, under
  // its weight-gradient MFMAs, the LDS stores after them (loads followed at once by their stores
  // exposed 1.3-2.7k clocks of load latency per step on the bottleneck group: 72.3 -> 70.0 us,
  // tools/var_specs/bstage.py r04v8)
  struct StRegs {
    uint4 nv[3];
    f32x4 nd2[ND2];
    uint32_t nmk;
  };
  auto stage_ld = [&](int fi, int fd, StRegs& r) {
    r.nmk = 0;
    if (fi >= 0) c1_load_frame<float>(x + rm.map(fi) * IMG, tid, r.nv);
    if (fd >= 0) {
      const float* src = dy2 + (size_t)fd * P2 * OC2;
#pragma unroll
      for (int i = 0; i < ND2; ++i) {
        const int e = tid + i * 256;
        r.nd2[i] = e < D2V ? *reinterpret_cast<const f32x4*>(src + e * 4) : F::zero();
      }
      if (tid < c1::NPIX) r.nmk = mask1[(size_t)fd * c1::NPIX + tid];
    }
  };
  auto stage_st = [&](int fi, int bi, int fd, int bd, const StRegs& r) {
    if (fd >= 0) {
      float* d2s = d2s_buf(bd);
#pragma unroll
      for (int i = 0; i < ND2; ++i) {
        const int e = tid + i * 256;
        if (e < D2V) *reinterpret_cast<f32x4*>(d2s + ((e * 4) / OC2) * LDD + (e * 4) % OC2) = r.nd2[i];
      }
      if (tid < c1::NPIX) msk_buf(bd)[tid] = r.nmk;
    }
    if (fi < 0) return;
    uint8_t* img = img_buf(bi);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int vi = tid + i * 256, ci = vi >> 8, yy = (vi & 255) >> 2, xq = vi & 3;
      const int Y = yy >> 2, bb = yy & 3;
      const uint32_t w[4] = {r.nv[i].x, r.nv[i].y, r.nv[i].z, r.nv[i].w};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint32_t t = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) t |= ((w[q] >> (8 * d)) & 255u) << (8 * q);
        *reinterpret_cast<uint32_t*>(img + (Y * c1::CH + ci * 16 + bb * 4 + d) * XP + 4 * xq) = t;
      }
    }
  };
  if (is_a && nF > 0 && load_w2) c12_load_w2(w2t, wb, wave, lane);
  // zero once: each half-Z tile's row 36, and the dY1 pad rows (ix = 15) of both buffers
  if (is_a && lane < OC1 / 2) *reinterpret_cast<f32x4*>(zw + P2 * LDZ + 4 * lane) = F::zero();
  for (int e = (int)threadIdx.x; e < 2 * H1 * (LDX / 4); e += 512) {
    const int b = e / (H1 * (LDX / 4)), r = e % (H1 * (LDX / 4));
    *reinterpret_cast<f32x4*>(dyt_buf(b) + ((r / (LDX / 4)) * 16 + 15) * LDX + 4 * (r % (LDX / 4))) = F::zero();
  }
  if (!is_a && nF > 0) stage(-1, 0, f0, 0);
  __syncthreads();
  // A: gather items of this lane: channels 4 cg .. 4 cg + 3 of class cells (qy, qx = slot)
  const int cg = lane & 7, slot = lane >> 3;
  // B: this wave's tap (ty, tx) of the conv1 weight gradient
  const int ty = wave >> 1, tx = wave & 1;
  // the groups run separate loops with the same barrier count (nF + 1), so that the compiler
  // keeps each group's loop-carried registers (A: the W2 fragments; B: the accumulators) apart
  if (is_a) {
    // the gather's Z chunk selectors: nibble d = cg ^ zswz(row) for rows = slot + d (mod 8)
    uint32_t zsel = 0;
#pragma unroll
    for (int d = 0; d < 8; ++d) zsel |= (uint32_t)(cg ^ L::zswz((slot + d) & 7)) << (4 * d);
    for (int it = 0; it < nF; ++it) {
      const int b = it & 1;
      // the gather's lane offsets recomputed per frame (not hoisted out of the loop as ~50 live
      // VGPRs)
      int sl = slot;
      uint32_t zt8 = zsel;
      asm volatile("" : "+v"(sl), "+v"(zt8));
      const float* d2s = d2s_buf(b);
      const uint32_t* msk = msk_buf(b);
      float* dyt = dyt_buf(b);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        __builtin_amdgcn_sched_barrier(0);  // one half's registers live at a time
        // ---- Z of taps 2 hf, 2 hf + 1 (Z^T tiles: A = the W2 fragments, rows = ci; B = the
        // dY2 rows, cols = op, read one k-step ahead), ops 32..35 on 4x4x1 blocks: block b =
        // 4 g + og (lane 16 g + 4 og + j) takes rows 4 og .. + 3 of W2 element e at k-phase
        // g = lane >> 4, op 32 + j; the k-phases summed by a fixed butterfly at the end ----
        f32x4 z[2][4];  // [op tile][tap 2 hf + (cc >> 1), ci tile cc & 1]
        f32x4 z4[4];    // ops 32..35, per cc
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) z[0][cc] = z[1][cc] = z4[cc] = f32x4{0.f, 0.f, 0.f, 0.f};
        V a2[2][3];
        auto a2load = [&](int ks, V* a) {
#pragma unroll
          for (int rt = 0; rt < 2; ++rt)
            a[rt] = *reinterpret_cast<const V*>(d2s + (16 * rt + (lane & 15)) * LDD + ks * KS + kl);
          a[2] = *reinterpret_cast<const V*>(d2s + (32 + (lane & 3)) * LDD + ks * KS + kl);
        };
#pragma unroll
        for (int ks = 0; ks < NKO; ++ks) {
          a2load(ks, a2[ks & 1]);
#pragma unroll
          for (int e = 0; e < F::NE; ++e) {
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
              for (int cc = 0; cc < 4; ++cc)
                z[rt][cc] = F::mma_e(e, wb[2 * hf + (cc >> 1)][ks][cc & 1], a2[ks & 1][rt], z[rt][cc]);
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
              z4[cc] = __builtin_amdgcn_mfma_f32_4x4x1f32(wb[2 * hf + (cc >> 1)][ks][cc & 1][e],
                                                         a2[ks & 1][2][e], z4[cc], 0, 0, 0);
          }
        }
        // the previous half's gather reads of the Z tile are done before it is overwritten
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
          const int op = 16 * rt + (lane & 15);
#pragma unroll
          for (int cc = 0; cc < 4; ++cc)
            *reinterpret_cast<f32x4*>(zw + op * LDZ + 4 * ((8 * (cc >> 1) + 4 * (cc & 1) + (kl >> 2)) ^
                                                          L::zswz(lane & 7))) = z[rt][cc];
        }
        {
          // the k-phase sums of the four cc at once: row cc of t holds cc's (rows_sum4), lane
          // 16 cc + 4 og + j stores ci 16 (cc & 1) + 4 og .. + 3 of op 32 + j
          f32x4 t;
#pragma unroll
          for (int q = 0; q < 4; ++q) t[q] = rows_sum4(z4[0][q], z4[1][q], z4[2][q], z4[3][q]);
          const int cc = lane >> 4;
          *reinterpret_cast<f32x4*>(zw + (32 + (lane & 3)) * LDZ +
                                    4 * ((8 * (cc >> 1) + 4 * (cc & 1) + ((lane >> 2) & 3)) ^
                                         L::zswz(32 + (lane & 3)))) = t;
        }
        // the wave's own Z stores are done before its gather reads them (LDS is in order per
        // wave; the wait + clobber keeps the compiler from moving the reads up)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // ---- col2im of class (py, px), taps (j1 = hf, j2): input pixel (2 qy + py, 2 qx + px)
        // adds tap (py + 2 hf, px + 2 j2) at dY2 cell (qy - hf, qx - j2), order j2.  Half 0
        // stores the partial sum, half 1 adds to it, masks, keeps the bias partials.  Branch-
        // free (an out-of-range tap reads the zero row), row qy + 1's reads in flight while row
        // qy is summed (two-stage pipeline pinned by scheduling barriers) ----
        f32x4 zt[2][3];
        uint32_t mk[2];
        auto gload = [&](int qy, f32x4* zz, uint32_t& m) {
          const int qx = sl, iy = 2 * qy + py, ix = 2 * qx + px;
          const bool pv = iy < H1 && ix < H1;
#pragma unroll
          for (int j2 = 0; j2 < 2; ++j2) {
            const int oy = qy - hf, ox = qx - j2;
            const bool ok = pv && oy >= 0 && oy < H2 && ox >= 0 && ox < H2;
            // chunk (8 j2 + cg) ^ zswz(row): row mod 8 = (sl + d) mod 8, nibble d of zt8
            const int d = (oy * H2 - j2) & 7;
            const int zc = (int)((zt8 >> (4 * d)) & 15u) ^ (8 * j2);
            zz[j2] = *reinterpret_cast<const f32x4*>(zw + (ok ? oy * H2 + ox : P2) * LDZ + 4 * zc);
          }
          if (hf == 1) {
            zz[2] = *reinterpret_cast<const f32x4*>(dyt + (pv ? iy * 16 + ix : 0) * LDX + 4 * cg);
            m = msk[pv ? iy * H1 + ix : 0];
          }
        };
        gload(0, zt[0], mk[0]);
#pragma unroll
        for (int qy = 0; qy < 8; ++qy) {
          if (qy + 1 < 8) gload(qy + 1, zt[(qy + 1) & 1], mk[(qy + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);
          const int qx = sl, iy = 2 * qy + py, ix = 2 * qx + px;
          const bool pv = iy < H1 && ix < H1;
          f32x4 v;
          if (hf == 0) {
            v = zt[qy & 1][0] + zt[qy & 1][1];
          } else {
            f32x4 sum = zt[qy & 1][2];
            sum += zt[qy & 1][0];
            sum += zt[qy & 1][1];
            // the ReLU mask as a bit mask: a sign-extended 1-bit field is 0 or ~0, so the AND
            // keeps the sum or makes +0 (a select, in two instructions instead of three)
            const uint32_t m = pv ? mk[qy & 1] : 0u;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              v[q] = (m >> (4 * cg + q)) & 1u ? sum[q] : 0.f;
              bsum[q] += v[q];
            }
          }
          // branch-free: a lane off the 15 x 15 grid holds v = +0 (its Z reads took the zero
          // row, its mask is 0) and stores it into pad row 15 (iy 0, ix 15), which stays zero
          *reinterpret_cast<f32x4*>(dyt + (pv ? iy * 16 + ix : 15) * LDX + 4 * cg) = v;
          __builtin_amdgcn_sched_barrier(0);
        }
        // half 1 reads back the partial sums this wave stored (LDS order per wave)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
    __syncthreads();
  } else {
    // group B stages every frame: in step k (after its weight gradient of frame k - 1), frame
    // k's image (read by B in step k + 1) and frame k + 1's dY2 / mask (read by A in step k + 1)
    stage(nF > 0 ? f0 : -1, 0, nF > 1 ? f0 + 1 : -1, 1);
    __syncthreads();
    for (int it = 1; it <= nF; ++it) {
      StRegs sr;
      stage_ld(it < nF ? f0 + it : -1, it + 1 < nF ? f0 + it + 1 : -1, sr);
      // ---- conv1 weight gradient of frame it - 1, as three exact bf16 MFMA passes: A = dY1
      // (rows oc, k = pixel) split exactly into hi + mid + lo bf16 terms (truncation: the top 8
      // significand bits of x, then of the remainder, then the <= 8 bits left -- each term's fp32
      // bits are its bf16 in the high half), B = the image bytes of cell (iy + ty, ix + tx),
      // channel n (exact in bf16).  Every product is the fp32 product; 16x16x32 bf16 MFMAs take
      // half the cycles of 16x16x4 f32 for 8x the K.  k-block kb = pixel rows 32 kb .. 32 kb + 31
      // (image rows 2 kb, 2 kb + 1); lane group g holds pixels 8 g .. 8 g + 7 of it: dY1 rows
      // (clamped to the 240 that exist) and 8 consecutive image bytes (funnel-shifted by tx).
      // The 16 pixels of image row 15 (kb = 7, g >= 2) are padding: their B operand is zero.
      // WKS: each wave takes two k-blocks of all four taps; else tap (ty, tx) = wave over all
      // eight k-blocks. ----
      const int b = (it - 1) & 1;
      const float* dyt = dyt_buf(b);
      const uint8_t* img = img_buf(b);
      using FB = Frag<__bf16>;
      typedef FB::vec VB;
      constexpr int NKB = 8;
      const int g = lane >> 4, col = lane & 15;
      // the high halves of two fp32 words as a bf16 pair (x0 low, x1 high)
      auto hi2 = [](uint32_t x0, uint32_t x1) { return __builtin_amdgcn_perm(x1, x0, 0x07060302u); };
      if constexpr (L::WKS) {
        // k-blocks kb = 2 wave, 2 wave + 1 of all four taps: per ty, image bytes X = 8 (g & 1)
        // .. + 8, converted once for both tx; padding pixels take zero image bytes
        struct Raw {
          float a[2][8];        // dY1 of oc 16 i + col, pixels 8 g .. 8 g + 7
          uint32_t w[2][3][3];  // [ty][channel tile j] image dwords at X = 8 (g & 1) + {0, 4, 8}
        };
        auto load = [&](int kb, Raw& r) {
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            const int pr = min(32 * kb + 8 * g + c, L::NROW - 1);
#pragma unroll
            for (int i = 0; i < 2; ++i) r.a[i][c] = dyt[pr * LDX + 16 * i + col];
          }
          const bool pad = kb == NKB - 1 && g >= 2;  // image row 15: zero bytes
#pragma unroll
          for (int ty = 0; ty < 2; ++ty) {
            const int Y = min(2 * kb + (g >> 1) + ty, c1::GRID - 1);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              const uint32_t* wp = reinterpret_cast<const uint32_t*>(img + (Y * c1::CH + 16 * j + col) * XP + 8 * (g & 1));
#pragma unroll
              for (int q = 0; q < 3; ++q) r.w[ty][j][q] = pad ? 0u : wp[q];
            }
          }
        };
        Raw rr[2];
        load(2 * wave, rr[0]);
        load(2 * wave + 1, rr[1]);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const Raw& r = rr[kk];  // k-block 2 wave + kk
          // A: the three terms of the 16 dY1 values (truncation: the top 8 significand bits of x,
          // then of the remainder, then the <= 8 bits left; each term's fp32 bits are its bf16 in
          // the high half, every product the fp32 product)
          VB fa[2][3];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            uint32_t th[4], tm[4], tl[4];
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
              uint32_t x[2], r1[2], r2[2];
#pragma unroll
              for (int u = 0; u < 2; ++u) {
                x[u] = __builtin_bit_cast(uint32_t, r.a[i][c + u]);
                const float f1 = r.a[i][c + u] - __builtin_bit_cast(float, x[u] & 0xffff0000u);
                r1[u] = __builtin_bit_cast(uint32_t, f1);
                r2[u] = __builtin_bit_cast(uint32_t, f1 - __builtin_bit_cast(float, r1[u] & 0xffff0000u));
              }
              th[c / 2] = hi2(x[0], x[1]);
              tm[c / 2] = hi2(r1[0], r1[1]);
              tl[c / 2] = hi2(r2[0], r2[1]);
            }
            fa[i][0] = __builtin_bit_cast(VB, th);
            fa[i][1] = __builtin_bit_cast(VB, tm);
            fa[i][2] = __builtin_bit_cast(VB, tl);
          }
#pragma unroll
          for (int ty = 0; ty < 2; ++ty) {
            // B of taps (ty, 0) and (ty, 1), one channel tile j at a time: image bytes X = 0 .. 8
            // (from 8 (g & 1)) -> fp32 (exact), pairs (X, X + 1) from X = tx as bf16 (the high
            // halves; exact for bytes)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              uint32_t f[9];
#pragma unroll
              for (int k = 0; k < 9; ++k)
                f[k] = __builtin_bit_cast(uint32_t, (float)((r.w[ty][j][k >> 2] >> (8 * (k & 3))) & 255u));
              VB fb[2];
#pragma unroll
              for (int tx = 0; tx < 2; ++tx) {
                uint32_t t[4];
#pragma unroll
                for (int p = 0; p < 4; ++p) t[p] = hi2(f[2 * p + tx], f[2 * p + tx + 1]);
                fb[tx] = __builtin_bit_cast(VB, t);
              }
#pragma unroll
              for (int tx = 0; tx < 2; ++tx)
#pragma unroll
                for (int tm = 0; tm < 3; ++tm)
#pragma unroll
                  for (int i = 0; i < 2; ++i)
                    acc[2 * ty + tx][i][j] = FB::mma(fa[i][tm], fb[tx], acc[2 * ty + tx][i][j]);
            }
          }
        }
      } else {
        struct Raw {
          float a[2][8];     // dY1 of oc 16 i + col, pixels 8 g .. 8 g + 7
          uint32_t w[3][3];  // image dwords at X = 8 (g & 1) + {0, 4, 8}, channel tile j
        };
        auto load = [&](int kb, Raw& r) {
  #pragma unroll
          for (int c = 0; c < 8; ++c) {
            const int pr = min(32 * kb + 8 * g + c, L::NROW - 1);
  #pragma unroll
            for (int i = 0; i < 2; ++i) r.a[i][c] = dyt[pr * LDX + 16 * i + col];
          }
          const int Y = min(2 * kb + (g >> 1) + ty, c1::GRID - 1);
  #pragma unroll
          for (int j = 0; j < 3; ++j) {
            const uint32_t* wp = reinterpret_cast<const uint32_t*>(img + (Y * c1::CH + 16 * j + col) * XP + 8 * (g & 1));
  #pragma unroll
            for (int q = 0; q < 3; ++q) r.w[j][q] = wp[q];
          }
        };
        Raw rr[2];
        load(0, rr[0]);
  #pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
          const Raw& r = rr[kb & 1];
          // A: the three terms of the 16 dY1 values
          VB fa[2][3];
  #pragma unroll
          for (int i = 0; i < 2; ++i) {
            uint32_t th[4], tm[4], tl[4];
  #pragma unroll
            for (int c = 0; c < 8; c += 2) {
              uint32_t x[2], r1[2], r2[2];
  #pragma unroll
              for (int u = 0; u < 2; ++u) {
                x[u] = __builtin_bit_cast(uint32_t, r.a[i][c + u]);
                const float f1 = r.a[i][c + u] - __builtin_bit_cast(float, x[u] & 0xffff0000u);
                r1[u] = __builtin_bit_cast(uint32_t, f1);
                r2[u] = __builtin_bit_cast(uint32_t, f1 - __builtin_bit_cast(float, r1[u] & 0xffff0000u));
              }
              th[c / 2] = hi2(x[0], x[1]);
              tm[c / 2] = hi2(r1[0], r1[1]);
              tl[c / 2] = hi2(r2[0], r2[1]);
            }
            fa[i][0] = __builtin_bit_cast(VB, th);
            fa[i][1] = __builtin_bit_cast(VB, tm);
            fa[i][2] = __builtin_bit_cast(VB, tl);
          }
          // B: 8 image bytes per channel tile -> bf16 (exact), zero on the padding row
          const bool pad = kb == NKB - 1 && g >= 2;
          VB fb[3];
  #pragma unroll
          for (int j = 0; j < 3; ++j) {
            const uint32_t w0 = __builtin_amdgcn_alignbyte(r.w[j][1], r.w[j][0], tx);
            const uint32_t w1 = __builtin_amdgcn_alignbyte(r.w[j][2], r.w[j][1], tx);
            uint32_t t[4];
  #pragma unroll
            for (int h = 0; h < 2; ++h) {
              const uint32_t w = h ? w1 : w0;
              const uint32_t f0 = __builtin_bit_cast(uint32_t, (float)(w & 255u));
              const uint32_t f1 = __builtin_bit_cast(uint32_t, (float)((w >> 8) & 255u));
              const uint32_t f2 = __builtin_bit_cast(uint32_t, (float)((w >> 16) & 255u));
              const uint32_t f3 = __builtin_bit_cast(uint32_t, (float)(w >> 24));
              t[2 * h] = pad ? 0u : hi2(f0, f1);
              t[2 * h + 1] = pad ? 0u : hi2(f2, f3);
            }
            fb[j] = __builtin_bit_cast(VB, t);
          }
          if (kb + 1 < NKB) load(kb + 1, rr[(kb + 1) & 1]);
  #pragma unroll
          for (int tm = 0; tm < 3; ++tm)
  #pragma unroll
            for (int j = 0; j < 3; ++j)
  #pragma unroll
              for (int i = 0; i < 2; ++i) acc[0][i][j] = FB::mma(fa[i][tm], fb[j], acc[0][i][j]);
        }
      }
      stage_st(it < nF ? f0 + it : -1, it & 1, it + 1 < nF ? f0 + it + 1 : -1, (it + 1) & 1, sr);
      __syncthreads();
    }
  }
  // conv1 bias: group A's 32 lanes of each channel group (8 per wave, 4 waves) in a fixed order
  float* bred = smem + L::Z0;
  if (is_a) *reinterpret_cast<f32x4*>(bred + 4 * tid) = f32x4{bsum[0], bsum[1], bsum[2], bsum[3]};
  // WKS: group B's k-block partials of every tap -> the image / dY1 tiles' space (free now)
  f32x4* wpart = reinterpret_cast<f32x4*>(smem + L::IMG);
  static_assert(!L::WKS || 4 * 4 * 6 * 64 * 4 <= L::D2S - L::IMG, "partials fit");
  if constexpr (L::WKS) {
    if (!is_a) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) wpart[((wave * 4 + t) * 6 + 3 * i + j) * 64 + lane] = acc[t][i][j];
    }
  }
  __syncthreads();
  if (is_a && tid < OC1) {
    float bs = 0.f;
#pragma unroll 8
    for (int s = 0; s < 32; ++s) bs += bred[4 * (s * 8 + (tid >> 2)) + (tid & 3)];
    slab_bias[(size_t)wg * OC1 + tid] = bs;
  }
  if (!is_a) {
    // wave w writes tap w (WKS: the four waves' k-block partials of it, summed in wave order)
    if constexpr (L::WKS) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          f32x4 v = wpart[((0 * 4 + wave) * 6 + 3 * i + j) * 64 + lane];
#pragma unroll
          for (int w = 1; w < 4; ++w) v += wpart[((w * 4 + wave) * 6 + 3 * i + j) * 64 + lane];
          acc[0][i][j] = v;
        }
    }
    const size_t so = (size_t)wg * OC1 * K1;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int col = wave * c1::CH + 16 * j + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          slab[so + (size_t)(16 * i + 4 * (lane >> 4) + q) * K1 + col] = acc[0][i][j][q] * (1.f / 255.f);
      }
  }
}

template <typename T, class O = ObsDirect>
DEV void conv12_bwd_body(const uint8_t* __restrict__ x, const T* __restrict__ w2,
                         const T* __restrict__ w2t, const T* __restrict__ dy2, const uint32_t* __restrict__ mask1,
                         float* __restrict__ slab, float* __restrict__ slab_bias, int N, int fpw,
                         int wg, char* __restrict__ lds, const O& rm = O{}) {
  if constexpr (sizeof(T) == 4) {  // fp32: the scatter-form body above
    Frag<float>::vec wb[4][OC2 / Frag<float>::KSTEP][2];
    conv12_bwd_body_f32<-1, O>(x, reinterpret_cast<const float*>(w2t), reinterpret_cast<const float*>(dy2),
                            mask1, slab, slab_bias, N, fpw, wg, lds, wb, true, rm);
    return;
  }
  using F = Frag<T>;
  typedef typename F::vec V;
  constexpr int KPL = F::KPL, KS = F::KSTEP;
  constexpr int LDI = c1::LB<T>::LDI;
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int LDX = c1::LB<T>::LDX;                 // dY1 tile row (elements)
  constexpr int LD2 = c1::LB<T>::LD2;                 // dY2 cell row (elements)
  constexpr int IMGSZ = c1::GRID * c1::GRID * LDI, DYSZ = c1::NPAD * LDX;
  constexpr int D2V = P2 * OC2 / VEC;                 // 16-byte vectors of one dY2 frame
  constexpr int ND2 = (D2V + 255) / 256;
  constexpr int NOK = OC2 / KS;                       // k-steps per tap
  constexpr int G = c12_groups<T>();
  constexpr int GSZ = IMGSZ + DYSZ + c12::NCELL * LD2;  // elements of one group's tiles
  static_assert(GSZ == C12BLds<T>::GSZ, "LDS layout");
  T* smem = reinterpret_cast<T*>(lds);
  uint32_t (*msk_all)[c1::NPIX] = reinterpret_cast<uint32_t (*)[c1::NPIX]>(lds + C12BLds<T>::MSK);
  float* bred = reinterpret_cast<float*>(lds + C12BLds<T>::BRED);
  const int grp = threadIdx.x >> 8, tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  T* img = smem + grp * GSZ;
  T* dyt = img + IMGSZ;
  T* d2s = dyt + DYSZ;
  uint32_t* msk = msk_all[grp];
  const int f0 = wg * fpw, f1 = min(N, f0 + fpw);
  f32x4 acc[2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};  // conv1 bias partials
  uint4 nv[3];
  V nd2[ND2];
  uint32_t nmk = 0;
  auto fetch = [&](int f) {
    c1_load_frame<T>(x + rm.map(f) * IMG, tid, nv);
    const T* src = dy2 + (size_t)f * P2 * OC2;
#pragma unroll
    for (int i = 0; i < ND2; ++i) {
      const int e = tid + i * 256;
      nd2[i] = e < D2V ? *reinterpret_cast<const V*>(src + e * VEC) : F::zero();
    }
    if (tid < c1::NPIX) nmk = mask1[(size_t)f * c1::NPIX + tid];
  };
  if (f0 + grp < f1) fetch(f0 + grp);  // the first frame is in flight during the prologue
  // class of this wave: output pixels iy = 2 qy + py, ix = 2 qx + px; taps kh = py + 2 j1,
  // kw = px + 2 j2 read dY2 at (qy - j1, qx - j2)
  const int py = wave >> 1, px = wave & 1;
  V wa[4][2][NOK];  // [tap j1*2+j2][ci tile][k-step]: A[ci][oc] = W2[oc][kh][kw][ci]
  if constexpr (sizeof(T) == 2) {
    // bf16: W2 [64][512] staged through LDS with 16-byte loads (rows padded to 528 and stored
    // bit-2/3 swapped, wg_row), the fragments (k = oc along the lane's 8 values) read with the
    // transposing LDS read, conflict-free
    constexpr int LDW = K2 + 2 * VEC, NWV = OC2 * K2 / VEC, NT = 256 * G, NPT = NWV / NT;
    static_assert(NWV % NT == 0 && OC2 * LDW <= G * GSZ, "w2 staging");
    T* w2s = smem;
    V wv[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = (int)threadIdx.x + i * NT;
      wv[i] = *reinterpret_cast<const V*>(w2 + (size_t)e * VEC);
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = (int)threadIdx.x + i * NT, row = e / (K2 / VEC), c = (e % (K2 / VEC)) * VEC;
      *reinterpret_cast<V*>(w2s + wg_row(row) * LDW + c) = wv[i];
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int kh = py + 2 * (t >> 1), kw = px + 2 * (t & 1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int ks = 0; ks < NOK; ++ks)
          wa[t][i][ks] = lds_frag_k_sw(w2s + ks * KS * LDW + (kh * KS2 + kw) * OC1 + 16 * i, LDW, lane);
    }
    __syncthreads();  // the staging area becomes the frame tiles
  } else {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int kh = py + 2 * (t >> 1), kw = px + 2 * (t & 1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int ks = 0; ks < NOK; ++ks) {
          const T* src = w2 + (size_t)(ks * KS + KPL * (lane >> 4)) * K2 + (kh * KS2 + kw) * OC1 +
                         16 * i + (lane & 15);
          V v;
#pragma unroll
          for (int j = 0; j < KPL; ++j) v[j] = src[(size_t)j * K2];
          wa[t][i][ks] = v;
        }
    }
  }
  // zero the dY1 rows no pixel writes and the dY2 cell grid once (the border stays zero);
  // the dY1 rows in 4-element pieces (rows of 36 elements start 8-byte aligned).  bf16: dY1
  // rows are grid rows oy * 16 + ox (the s2d image's), so the pad rows are ox = 15 and
  // oy = 15; fp32: rows are pixels, pad rows 225..255.
  static_assert((c1::NPAD - c1::NPIX) * LDX % 4 == 0 && c12::NCELL * LD2 % VEC == 0 &&
                c1::NPIX * LDX % 4 == 0 && LDX % 4 == 0, "zero fill");
  constexpr bool GR = sizeof(T) == 2;
  for (int e = tid; e < (c1::NPAD - c1::NPIX) * LDX / 4; e += 256) {
    const float z[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (GR) {
      const int rr = e / (LDX / 4), c = (e % (LDX / 4)) * 4;
      const int row = rr < H1 ? rr * c1::GRID + H1 : c1::GRID * H1 + (rr - H1);
      store4(dyt + row * LDX + c, z);
    } else {
      store4(dyt + c1::NPIX * LDX + e * 4, z);
    }
  }
  for (int e = tid; e < c12::NCELL * LD2 / VEC; e += 256)
    *reinterpret_cast<V*>(d2s + e * VEC) = F::zero();
  const int tapoff = ((wave >> 1) * c1::GRID + (wave & 1)) * LDI;
  const int kl = KPL * (lane >> 4);
  const int n_it = (f1 - f0 + G - 1) / G;
  for (int it = 0; it < n_it; ++it) {
    const int f = f0 + G * it + grp;
    const bool active = f < f1;
    __syncthreads();  // the previous frame's readers are done
    if (active) {
    c1_stash_frame<T, LDI>(img, tid, nv);
#pragma unroll
    for (int i = 0; i < ND2; ++i) {
      const int e = tid + i * 256;
      if (e < D2V) {
        const int cell = (e * VEC) / OC2, oc = (e * VEC) % OC2;
        const int oy = cell / H2, ox = cell - oy * H2;
        *reinterpret_cast<V*>(d2s + ((oy + 1) * c12::QG + ox + 1) * LD2 + oc) = nd2[i];
      }
    }
    if (tid < c1::NPIX) msk[tid] = nmk;
    }
    __syncthreads();
    if (f + G < f1) fetch(f + G);
    // ---- conv2 dgrad of class `wave` -> masked dY1 rows in LDS (+ conv1 bias partials) ----
    // Only the tap-(0,0) B fragments are read from LDS (cells (qy, qx) of all 4 column tiles);
    // the shifted taps are lane moves: the 16 lanes of a fragment row are cells qx = l & 7 of
    // rows qy = 2 nt + ((l >> 3) & 1), so qx - 1 is a DPP row shift right by one (zero in at
    // qx = 0: lane 7 -> 8 carries the always-zero column qx = 7) and qy - 1 is a shift by 8,
    // taking the lower half from the previous tile.
    if (active) {
      V b0[4][NOK];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int cell = nt * 16 + (lane & 15), qy = cell >> 3, qx = cell & 7;
        const T* brow = d2s + ((qy + 1) * c12::QG + qx + 1) * LD2 + kl;
#pragma unroll
        for (int ks = 0; ks < NOK; ++ks) b0[nt][ks] = *reinterpret_cast<const V*>(brow + ks * KS);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {  // 16-cell column tiles of the 8x8 class grid
        f32x4 d[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int ks = 0; ks < NOK; ++ks) {
          const V bt0 = b0[nt][ks];
          const V bt1 = dpp_move<0x111>(bt0);                       // (qy, qx - 1)
          V bt2 = dpp_move<0x118>(bt0);                             // (qy - 1, qx): odd rows
          if (nt > 0) bt2 = vor(bt2, dpp_move<0x108>(b0[nt - 1][ks]));  // even rows
          const V bt3 = dpp_move<0x111>(bt2);                       // (qy - 1, qx - 1)
          d[0] = F::mma(wa[0][0][ks], bt0, d[0]);
          d[1] = F::mma(wa[0][1][ks], bt0, d[1]);
          d[0] = F::mma(wa[1][0][ks], bt1, d[0]);
          d[1] = F::mma(wa[1][1][ks], bt1, d[1]);
          d[0] = F::mma(wa[2][0][ks], bt2, d[0]);
          d[1] = F::mma(wa[2][1][ks], bt2, d[1]);
          d[0] = F::mma(wa[3][0][ks], bt3, d[0]);
          d[1] = F::mma(wa[3][1][ks], bt3, d[1]);
        }
        const int cell = nt * 16 + (lane & 15), qy = cell >> 3, qx = cell & 7;
        const int iy = 2 * qy + py, ix = 2 * qx + px;
        if (iy < H1 && ix < H1) {
          const int p = iy * H1 + ix, drow = GR ? iy * c1::GRID + ix : p;
          const uint32_t m = msk[p];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int ci = 16 * i + 4 * (lane >> 4);
            float v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              v[q] = (m >> (ci + q)) & 1u ? d[i][q] : 0.f;
              bsum[i][q] += v[q];
            }
            store4(dyt + drow * LDX + ci, v);
          }
        }
      }
    }
    __syncthreads();  // (every group reaches it: no early exit for an idle group)
    if (!active) continue;
    // ---- conv1 weight gradient: reduction over the frame's (padded) 256 pixels, fragments
    // software-pipelined one k-step ahead.  bf16: the k slots of a 32-deep step are the 32
    // grid rows kk .. kk + 31 taken in the order that gives each 32-lane half of a
    // transposing read 8 rows R + 4m (m = 0..7): at dY1's 18-dword and the image's 26-dword
    // row steps those are 8 disjoint 8-dword bank ranges (tools/ldsbank.py: dY1 reads 2.0x ->
    // 1.0x, image reads 1.88x -> 1.09x).  Rows without a pixel hold dY1 = 0; their image row
    // is clamped to the last pixel row (238) so that the tap offsets stay inside the stashed image
    // rows 0..255 (a 0 x NaN from an unwritten row would poison the sum). ----
    auto frag = [&](int kk, V* a, V* b) {
      if constexpr (sizeof(T) == 2) {
        const int g = lane >> 4, ii = lane & 15, q = ii >> 2, pp = ii & 3;
        const int r0 = kk + 4 * (q + 4 * (g & 1)) + 2 * (g >> 1);  // rows r0 (k 0..3), r0 + 1
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const bf16x4_t u = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(dyt + r0 * LDX + 16 * i + 4 * pp));
          const bf16x4_t w = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(dyt + (r0 + 1) * LDX + 16 * i + 4 * pp));
          V v;
          v[0] = u[0]; v[1] = u[1]; v[2] = u[2]; v[3] = u[3];
          v[4] = w[0]; v[5] = w[1]; v[6] = w[2]; v[7] = w[3];
          a[i] = v;
        }
        constexpr int RMAX = c1::GRID * (H1 - 1) + H1 - 1;  // 238: the last pixel row (+ 17 < 256)
        const int ra = min(r0, RMAX) * LDI + tapoff + 4 * pp;
        const int rb = min(r0 + 1, RMAX) * LDI + tapoff + 4 * pp;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const bf16x4_t u = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + ra + 16 * j));
          const bf16x4_t w = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + rb + 16 * j));
          V v;
          v[0] = u[0]; v[1] = u[1]; v[2] = u[2]; v[3] = u[3];
          v[4] = w[0]; v[5] = w[1]; v[6] = w[2]; v[7] = w[3];
          b[j] = v;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = lds_frag_k(dyt + kk * LDX + 16 * i, LDX, lane);
        const int g = lane >> 4, col = lane & 15;
        int rr[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          rr[jj] = c1_row(min(kk + 4 * g + jj, c1::NPIX - 1), 0) * LDI + tapoff + col;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          V v;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) v[jj] = (float)img[rr[jj] + 16 * j];
          b[j] = v;
        }
      }
    };
    constexpr int NKK = c1::NPAD / KS;
    V fa[2][2], fb[2][3];
    frag(0, fa[0], fb[0]);
#pragma unroll
    for (int s2 = 0; s2 < NKK; ++s2) {
      if (s2 + 1 < NKK) frag((s2 + 1) * KS, fa[(s2 + 1) & 1], fb[(s2 + 1) & 1]);
#pragma unroll
      for (int e = 0; e < F::NE; ++e)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) acc[i][j] = F::mma_e(e, fa[s2 & 1][i], fb[s2 & 1][j], acc[i][j]);
    }
  }
  // conv1 bias: sum each lane's partials over the 16 lanes of its channel group (fixed
  // butterfly order), then over the 4 class waves and the G groups in LDS, in a fixed order
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = bsum[i][q];
      v = row16_sum(v);
      bsum[i][q] = v;
    }
  __syncthreads();  // all groups are done with their tiles
  if ((lane & 15) == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) bred[(grp * 4 + wave) * OC1 + 16 * i + 4 * (lane >> 4) + q] = bsum[i][q];
  }
  // fixed-order combine of the groups' weight-gradient partials: group g > 0 -> LDS -> group 0
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int g = 1; g < G; ++g) {
    __syncthreads();
    if (grp == g) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) red[((i * 3 + j) * 4 + q) * 256 + tid] = acc[i][j][q];
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[i][j][q] += red[((i * 3 + j) * 4 + q) * 256 + tid];
    }
  }
  __syncthreads();
  if (grp != 0) return;
  if (tid < OC1) {
    float bs = 0.f;
#pragma unroll
    for (int g = 0; g < 4 * G; ++g) bs += bred[g * OC1 + tid];
    slab_bias[(size_t)wg * OC1 + tid] = bs;
  }
  const size_t so = (size_t)wg * OC1 * K1;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int col = wave * c1::CH + 16 * j + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        slab[so + (size_t)(16 * i + 4 * (lane >> 4) + q) * K1 + col] = acc[i][j][q] * (1.f / 255.f);
    }
}

template <typename T>
__global__ __launch_bounds__(256 * c12_groups<T>()) void conv12_bwd_s2d(const uint8_t* __restrict__ x,
                                                      const T* __restrict__ w2,     // [64][512]
                                                      const T* __restrict__ w2t,    // [512][64] (fp32)
                                                      const T* __restrict__ dy2,    // [N][36][64]
                                                      const uint32_t* __restrict__ mask1,  // [N][225]
                                                      float* __restrict__ slab,
                                                      float* __restrict__ slab_bias, int N,
                                                      int fpw) {
  __shared__ __attribute__((aligned(16))) char lds[C12BLds<T>::BYTES];
  conv12_bwd_body<T>(x, w2, w2t, dy2, mask1, slab, slab_bias, N, fpw, (int)blockIdx.x, lds);
}
