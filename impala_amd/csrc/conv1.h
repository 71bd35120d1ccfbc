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
template <typename T>
DEV void c1_stash_frame(T* img, int tid, const uint4 v[3]) {
  constexpr int LDI = c1::L<T>::LDI;
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

// ---------------------------------------------------------------------------------------
// forward: act1[n][p][oc] = relu(sum W'[oc][k'] s2d * 1/255 + b1), weights in registers.
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void conv1_fwd_s2d(const uint8_t* __restrict__ x,
                                                     const T* __restrict__ w,  // [32][192] k'
                                                     const float* __restrict__ bias,
                                                     T* __restrict__ out, int N) {
  using F = Frag<T>;
  typedef typename F::vec V;
  constexpr int LDI = c1::L<T>::LDI;
  constexpr int NKS = K1 / F::KSTEP;  // 6 (bf16) / 12 (f32)
  __shared__ __attribute__((aligned(16))) T img[c1::GRID * c1::GRID * LDI];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kl = F::KPL * (lane >> 4);
  V wa[2][NKS];  // A fragments: rows oc = 16*i + (lane & 15), all of K
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      wa[i][ks] = F::load(w + (16 * i + (lane & 15)) * K1 + ks * F::KSTEP + kl);
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
    c1_stash_frame<T>(img, tid, nv);
    __syncthreads();
    if (f + (int)gridDim.x < N) c1_load_frame<T>(x + (size_t)(f + gridDim.x) * IMG, tid, nv);
    for (int tile = wave; tile < 15; tile += 4) {  // 15 x 16 pixel tiles cover the 225 pixels
      const int p = min(tile * 16 + (lane & 15), c1::NPIX - 1);
      const int base = c1_row(p, 0) * LDI;
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int k = ks * F::KSTEP + kl, tap = k / c1::CH, ch = k - tap * c1::CH;
        const int off = ((tap >> 1) * c1::GRID + (tap & 1)) * LDI + ch;
        const V b = *reinterpret_cast<const V*>(img + base + off);
        acc[0] = F::mma(wa[0][ks], b, acc[0]);
        acc[1] = F::mma(wa[1][ks], b, acc[1]);
      }
      const int pc = tile * 16 + (lane & 15);
      if (pc < c1::NPIX) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = fmaxf(acc[i][q] * (1.f / 255.f) + bb[i][q], 0.f);
          store4(out + ((size_t)f * c1::NPIX + pc) * OC1 + 16 * i + 4 * (lane >> 4), v);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// weight gradient: dW'[oc][k'] = sum_{frames, p} dY[p][oc] * s2d[row(p, tap)][ch]  (1/255 at
// the end), reduction over the 225 (padded 256) pixels of each frame.  Wave w owns tap w
// (48 channels = 3 column tiles) for both 16-row oc tiles.  The workgroup handles a
// contiguous run of frames and writes one fp32 partial slab [32][192] (k' order) + bias sums.
// ---------------------------------------------------------------------------------------
template <typename T> constexpr int c1_wgrad_groups() { return sizeof(T) == 2 ? 2 : 1; }

template <typename T>
__global__ __launch_bounds__(256 * c1_wgrad_groups<T>()) void conv1_wgrad_s2d(const uint8_t* __restrict__ x,
                                                       const T* __restrict__ dy,  // [N][225][32]
                                                       float* __restrict__ slab,
                                                       float* __restrict__ slab_bias, int N,
                                                       int fpw) {
  // two 4-wave groups per workgroup work on alternating frames of the workgroup's run (two
  // frames in flight per CU on top of the one-frame register prefetch); their accumulators are
  // summed in a fixed order at the end.
  using F = Frag<T>;
  typedef typename F::vec V;
  constexpr int LDI = c1::L<T>::LDI;
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int LDX = OC1 + VEC;                      // dY tile row (elements)
  constexpr int DYV = c1::NPIX * OC1 / VEC;           // 16-byte vectors per dY frame
  constexpr int NDY = (DYV + 255) / 256;
  constexpr int IMGSZ = c1::GRID * c1::GRID * LDI, DYSZ = c1::NPAD * LDX;
  constexpr int G = c1_wgrad_groups<T>();
  __shared__ __attribute__((aligned(16))) T smem[G * (IMGSZ + DYSZ)];
  const int grp = threadIdx.x >> 8, tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  T* img = smem + grp * (IMGSZ + DYSZ);
  T* dyt = img + IMGSZ;
  const int f0 = blockIdx.x * fpw, f1 = min(N, f0 + fpw);
  // zero the padding rows 225..255 of the dY tile once (never overwritten)
  for (int e = tid; e < (c1::NPAD - c1::NPIX) * LDX; e += 256) dyt[c1::NPIX * LDX + e] = (T)0.f;
  f32x4 acc[2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bias_acc = 0.f;
  uint4 nv[3];
  V ndy[NDY];
  auto fetch = [&](int f) {
    c1_load_frame<T>(x + (size_t)f * IMG, tid, nv);
    const T* src = dy + (size_t)f * c1::NPIX * OC1;
#pragma unroll
    for (int i = 0; i < NDY; ++i) {
      const int e = tid + i * 256;
      ndy[i] = e < DYV ? *reinterpret_cast<const V*>(src + e * VEC) : F::zero();
    }
  };
  if (f0 + grp < f1) fetch(f0 + grp);
  const int tapoff = ((wave >> 1) * c1::GRID + (wave & 1)) * LDI;
  const int n_it = (f1 - f0 + G - 1) / G;
  for (int it = 0; it < n_it; ++it) {
    const int f = f0 + G * it + grp;
    const bool active = f < f1;
    __syncthreads();
    if (active) {
      c1_stash_frame<T>(img, tid, nv);
#pragma unroll
      for (int i = 0; i < NDY; ++i) {
        const int e = tid + i * 256;
        if (e < DYV) {
          const int row = (e * VEC) / OC1, col = (e * VEC) % OC1;
          *reinterpret_cast<V*>(dyt + row * LDX + col) = ndy[i];
        }
      }
    }
    __syncthreads();
    if (f + G < f1) fetch(f + G);
    if (!active) continue;
    {  // bias: 8 row groups x 32 channels, partial sums kept per thread across frames
      const int oc = tid & 31, rg = tid >> 5;
      float s0 = 0.f, s1 = 0.f;
      int r = rg;
      for (; r + 8 < c1::NPIX; r += 16) {
        s0 += (float)dyt[r * LDX + oc];
        s1 += (float)dyt[(r + 8) * LDX + oc];
      }
      if (r < c1::NPIX) s0 += (float)dyt[r * LDX + oc];
      bias_acc += s0 + s1;
    }
#pragma unroll 2
    for (int kk = 0; kk < c1::NPAD; kk += F::KSTEP) {
      V a[2], b[3];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = lds_frag_k(dyt + kk * LDX + 16 * i, LDX, lane);
      if constexpr (sizeof(T) == 2) {
        const int g = lane >> 4, ii = lane & 15, q = ii >> 2, pp = ii & 3;
        const int ra = c1_row(min(kk + 8 * g + q, c1::NPIX - 1), 0) * LDI + tapoff + 4 * pp;
        const int rb = c1_row(min(kk + 8 * g + 4 + q, c1::NPIX - 1), 0) * LDI + tapoff + 4 * pp;
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
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = F::mma(a[i], b[j], acc[i][j]);
    }
  }
  // fixed-order combine: group 1 -> LDS -> group 0; bias row groups likewise
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  if (G > 1 && grp == 1) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[((i * 3 + j) * 4 + q) * 256 + tid] = acc[i][j][q];
    red[24 * 256 + tid] = bias_acc;
  }
  __syncthreads();
  if (G > 1 && grp == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][j][q] += red[((i * 3 + j) * 4 + q) * 256 + tid];
    bias_acc += red[24 * 256 + tid];
  }
  __syncthreads();
  if (grp == 0) red[tid] = bias_acc;
  __syncthreads();
  if (grp != 0) return;
  if (tid < OC1) {
    float bsum = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) bsum += red[g * 32 + tid];
    slab_bias[(size_t)blockIdx.x * OC1 + tid] = bsum;
  }
  const size_t so = (size_t)blockIdx.x * OC1 * K1;
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
