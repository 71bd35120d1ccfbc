// Operand definitions plugged into gemm_rc / gemm_wg for each layer of the step.
// Activations are channels-last (pixel-major, channel-contiguous); frame n = b*T + t
// (batch-major flatten of agents/impala/learning.py:143).
#pragma once
#include "gemm.h"
#include "lnorm.h"
#include "net.h"

using namespace net;

// ------------------------------- forward ------------------------------------------------
// conv1: rows oc (32), cols pixel (n, oh, ow) in N*225, k = ci*64 + kh*8 + kw over u8 NCHW
// input (the x/255 of models/models.py:73 is folded into the epilogue: raw bytes are exact
// in bf16).  Epilogue: *1/255 + bias, ReLU -> act1[n][oh][ow][oc].
template <typename T> struct Conv1Fwd {
  static constexpr bool A_KMAJOR = false;
  static constexpr bool TILE_EPI = false;
  static constexpr int K = K1;
  int C;
  const T* w;
  const float* b;
  const uint8_t* x;
  T* out;
  struct ColCtx { const uint8_t* p; };
  DEV ColCtx col_ctx(int c) const {
    const int n = c / P1, p = c - n * P1, oh = p / H1, ow = p - oh * H1;
    return ColCtx{x + (size_t)n * IMG + (ST1 * oh) * H0 + ST1 * ow};
  }
  DEV const T* a_row(int r, int) const { return w + r * K; }
  DEV typename Frag<T>::vec load_b(const ColCtx& cc, int k) const {
    const int ci = k >> 6, kh = (k >> 3) & 7, kw = k & 7;
    const uint8_t* p = cc.p + ci * (H0 * H0) + kh * H0 + kw;
    if constexpr (sizeof(T) == 4) {
      return Frag<float>::from_u8(*reinterpret_cast<const uint32_t*>(p));
    } else {
      return Frag<__bf16>::from_u8_2(*reinterpret_cast<const uint32_t*>(p),
                                     *reinterpret_cast<const uint32_t*>(p + 4));
    }
  }
  DEV void store(int r, int c, float v[4]) const {
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = fmaxf(v[i] * (1.f / 255.f) + b[r + i], 0.f);
    store4(out + (size_t)c * OC1 + r, o);
  }
};

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
  DEV void store(int r, int c, float v[4]) const {
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = fmaxf(v[i] + b[r + i], 0.f);
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
  DEV void store(int r, int c, float v[4]) const {
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = fmaxf(v[i] + b[r + i], 0.f);
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
  float* z;  // pre-activation (fp32, kept for the GELU backward)
  T* h;
  struct ColCtx { const T* p; };
  DEV ColCtx col_ctx(int c) const { return ColCtx{y + (size_t)c * FLAT}; }
  DEV const T* a_row(int r, int) const { return w + r * K; }
  DEV typename Frag<T>::vec load_b(const ColCtx& cc, int k) const { return Frag<T>::load(cc.p + k); }
  DEV void store(int r, int c, float v[4]) const {
    float zz[4], hh[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      zz[i] = v[i] + b[r + i];
      hh[i] = gelu_f(zz[i]);
    }
    store4(z + (size_t)c * HID + r, zz);
    store4(h + (size_t)c * HID + r, hh);
  }
};

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
  DEV void tile_epilogue(const float* et, int ldt, int, int cc0, int tid) const {
    const int lane = tid & 63, wave = tid >> 6;
    const int frame = cc0 / P3 + wave;
    if ((frame + 1) * P3 > this->C) return;
    ln_frame_epilogue<T>(et + wave * P3 * ldt, ldt, frame, lane, this->b, gam, bet, this->out, y,
                         stats);
  }
};

// projection Linear + GELU + actor/critic heads fused: a 256(o) x 32(frame) tile holds whole
// h rows; the heads (16 x 256) are applied from LDS in the epilogue (wave 0..1: 16 frames each).
template <typename T> struct FcHeadsFwd : FcFwd<T> {
  static constexpr bool TILE_EPI = true;
  const T* wh;       // [16][256]
  const float* bh;   // [16]
  float* heads;      // [n][16]
  DEV void tile_epilogue(const float* et, int ldt, int, int cc0, int tid) const {
    // 1) z = acc + b, h = gelu(z): write z, h to HBM, h (fp32) back into the LDS tile
    float* etw = const_cast<float*>(et);
    for (int e = tid; e < 32 * (HID / 4); e += 256) {
      const int f = e / (HID / 4), r = (e % (HID / 4)) * 4;
      const int c = cc0 + f;
      float zz[4], hh[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        zz[k] = et[f * ldt + r + k] + this->b[r + k];
        hh[k] = gelu_f(zz[k]);
      }
      if (c < this->C) {
        store4(this->z + (size_t)c * HID + r, zz);
        store4(this->h + (size_t)c * HID + r, hh);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) etw[f * ldt + r + k] = (float)(T)hh[k];  // as stored (T)
    }
    __syncthreads();
    // 2) heads: out[f][o'] = sum_j wh[o'][j] h[f][j] + bh[o'], one 16x16 tile per wave 0..1
    const int lane = tid & 63, wave = tid >> 6;
    if (wave < 2) {
      using F = Frag<T>;
      const int kl = F::KPL * (lane >> 4);
      const int f = wave * 16 + (lane & 15);
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int k = 0; k < HID; k += F::KSTEP) {
        const typename F::vec a = F::load(wh + (lane & 15) * HID + k + kl);
        typename F::vec bv;
#pragma unroll
        for (int q = 0; q < F::KPL; ++q) bv[q] = (T)et[f * ldt + k + kl + q];
        acc = F::mma(a, bv, acc);
      }
      const int c = cc0 + f;
      if (c < this->C) {
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = acc[q] + bh[4 * (lane >> 4) + q];
        store4(heads + (size_t)c * HEADS + 4 * (lane >> 4), o);
      }
    }
  }
};

// ------------------------------- backward (dgrad) ---------------------------------------
// dh = dH . Wh  then GELU backward:  dz[n][j] = dh[n][j] * gelu'(z[n][j]).  K = 32 (padded).
template <typename T> struct HeadsDgrad {
  static constexpr bool A_KMAJOR = false;
  static constexpr bool TILE_EPI = false;
  static constexpr int K = HPAD;
  int C;
  const T* wt;  // [256][32]
  const T* dH;  // [n][32]
  const float* z;
  T* dz;
  struct ColCtx { const T* p; };
  DEV ColCtx col_ctx(int c) const { return ColCtx{dH + (size_t)c * HPAD}; }
  DEV const T* a_row(int r, int) const { return wt + r * K; }
  DEV typename Frag<T>::vec load_b(const ColCtx& cc, int k) const { return Frag<T>::load(cc.p + k); }
  DEV void store(int r, int c, float v[4]) const {
    float zz[4], o[4];
    load4(z + (size_t)c * HID + r, zz);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = v[i] * gelu_grad(zz[i]);
    store4(dz + (size_t)c * HID + r, o);
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
  DEV void store(int r, int c, float v[4]) const { store4(dy + (size_t)c * FLAT + r, v); }
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
  DEV void store(int r, int c, float v[4]) const {
    float a[4], o[4];
    load4(act + (size_t)c * OC2 + r, a);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = a[i] > 0.f ? v[i] : 0.f;
    store4(dx + (size_t)c * OC2 + r, o);
  }
};

// conv2 dgrad by stride-parity class (sub-pixel decomposition, no zero taps inside):
// cols = cls*NC + n*64 + iy'*8 + ix'  with ih = 2*iy' + py, iw = 2*ix' + px, cls = py*2+px;
// NC = N*64 rounded up to the tile width so no tile straddles two classes (columns
// q >= N*64 of a class are padding); rows ci (32); k = (j1*2+j2)*64 + oc with
// kh = py + 2*j1, kw = px + 2*j2, oh = iy' - j1.
// Epilogue applies conv1's ReLU mask (act1 > 0); ih/iw == 15 are outside the 15x15 map.
template <typename T> struct Conv2Dgrad {
  static constexpr bool A_KMAJOR = true;
  static constexpr bool TILE_EPI = false;
  static constexpr int K = 4 * OC2;
  int C;        // 4 * NC
  int NC;       // columns per class (multiple of the tile width)
  int NQ;       // valid columns per class = N * 64
  const T* w;   // w2 [64 oc][512 = (kh*4+kw)*32 + ci]; A[ci][t*64 + oc] read k-major
  const T* dy;  // dact2 [n][36][64]
  const T* act; // act1 (mask)
  T* dx;        // dact1
  struct ColCtx { const T* p; int iy, ix; };
  DEV ColCtx col_ctx(int c) const {
    const int cl = c / NC, q = min(c - cl * NC, NQ - 1), n = q >> 6, iy = (q >> 3) & 7, ix = q & 7;
    return ColCtx{dy + (size_t)n * P2 * OC2, iy, ix};
  }
  DEV const T* a_row(int, int) const { return nullptr; }
  DEV const T* a_kptr(int k, int r, int cw) const {
    const int cl = cw / NC, t = k >> 6, oc = k & 63;
    const int kh = (cl >> 1) + 2 * (t >> 1), kw = (cl & 1) + 2 * (t & 1);
    return w + (size_t)oc * K2 + (kh * KS2 + kw) * OC1 + r;
  }
  DEV typename Frag<T>::vec load_b(const ColCtx& cc, int k) const {
    const int t = k >> 6, oc = k & 63, j1 = t >> 1, j2 = t & 1;
    const int oy = cc.iy - j1, ox = cc.ix - j2;
    if (oy < 0 || oy >= H2 || ox < 0 || ox >= H2) return Frag<T>::zero();
    return Frag<T>::load(cc.p + (oy * H2 + ox) * OC2 + oc);
  }
  DEV void store(int r, int c, float v[4]) const {
    const int cl = c / NC, q = c - cl * NC;
    if (q >= NQ) return;
    const int n = q >> 6, iy = (q >> 3) & 7, ix = q & 7;
    const int ih = 2 * iy + (cl >> 1), iw = 2 * ix + (cl & 1);
    if (ih >= H1 || iw >= H1) return;
    const size_t o = ((size_t)(n * H1 + ih) * H1 + iw) * OC1 + r;
    float a[4], out[4];
    load4(act + o, a);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = a[i] > 0.f ? v[i] : 0.f;
    store4(dx + o, out);
  }
};

// ------------------------------- backward (wgrad) ---------------------------------------
// D[r][c] = sum_m X[m][r] * Y(m, c); X row-major [M][x_ld]; load_y returns 16 bytes of T
// (VEC consecutive c of one run: channels for conv2/3/FC/heads, kw for conv1).
template <typename T> struct HeadsWgrad {  // dWh[o'][j] = sum_n dH[n][o'] h[n][j]
  static constexpr int R = HEADS, C = HID;
  int M;
  float out_scale = 1.f;
  const T* x;  // dH [n][32]
  int x_ld = HPAD;
  const T* h;
  DEV const T* y_row(int m) const { return h + (size_t)m * HID; }
  DEV typename Frag<T>::vec load_y(const T* row, int c) const {
    return *reinterpret_cast<const typename Frag<T>::vec*>(row + c);
  }
};
template <typename T> struct FcWgrad {  // dWfc[o][j] = sum_n dz[n][o] y[n][j]
  static constexpr int R = HID, C = FLAT;
  int M;
  float out_scale = 1.f;
  const T* x;  // dz
  int x_ld = HID;
  const T* y;
  DEV const T* y_row(int m) const { return y + (size_t)m * FLAT; }
  DEV typename Frag<T>::vec load_y(const T* row, int c) const {
    return *reinterpret_cast<const typename Frag<T>::vec*>(row + c);
  }
};
template <typename T> struct Conv3Wgrad {  // m = (n, oy, ox) in N*16; c = (kh*3+kw)*64 + ci
  static constexpr int R = OC3, C = K3;
  int M;
  float out_scale = 1.f;
  const T* x;  // dact3
  int x_ld = OC3;
  const T* in;  // act2
  DEV const T* y_row(int m) const {  // top-left input pixel of the 3x3 patch
    const int n = m / P3, p = m - n * P3, oy = p / H3, ox = p - oy * H3;
    return in + ((size_t)(n * H2 + oy) * H2 + ox) * OC2;
  }
  DEV typename Frag<T>::vec load_y(const T* row, int c) const {
    const int tap = c >> 6, ci = c & 63, kh = tap / 3, kw = tap - kh * 3;
    return *reinterpret_cast<const typename Frag<T>::vec*>(row + (kh * H2 + kw) * OC2 + ci);
  }
};
template <typename T> struct Conv2Wgrad {  // m = (n, oy, ox) in N*36; c = (kh*4+kw)*32 + ci
  static constexpr int R = OC2, C = K2;
  int M;
  float out_scale = 1.f;
  const T* x;  // dact2
  int x_ld = OC2;
  const T* in;  // act1
  DEV const T* y_row(int m) const {
    const int n = m / P2, p = m - n * P2, oy = p / H2, ox = p - oy * H2;
    return in + ((size_t)(n * H1 + ST2 * oy) * H1 + ST2 * ox) * OC1;
  }
  DEV typename Frag<T>::vec load_y(const T* row, int c) const {
    const int tap = c >> 5, ci = c & 31, kh = tap >> 2, kw = tap & 3;
    return *reinterpret_cast<const typename Frag<T>::vec*>(row + (kh * H1 + kw) * OC1 + ci);
  }
};
template <typename T> struct Conv1Wgrad {  // m = (n, oy, ox) in N*225; c = ci*64 + kh*8 + kw
  static constexpr int R = OC1, C = K1;
  int M;
  float out_scale = 1.f / 255.f;
  const T* x;  // dact1
  int x_ld = OC1;
  const uint8_t* img;
  DEV const uint8_t* y_row(int m) const {
    const int n = m / P1, p = m - n * P1, oy = p / H1, ox = p - oy * H1;
    return img + (size_t)n * IMG + (ST1 * oy) * H0 + ST1 * ox;
  }
  DEV typename Frag<T>::vec load_y(const uint8_t* row, int c) const {
    const int ci = c >> 6, kh = (c >> 3) & 7, kw = c & 7;
    const uint8_t* q = row + ci * (H0 * H0) + kh * H0 + kw;
    if constexpr (sizeof(T) == 4) {
      return Frag<float>::from_u8(*reinterpret_cast<const uint32_t*>(q));
    } else {
      return Frag<__bf16>::from_u8_2(*reinterpret_cast<const uint32_t*>(q),
                                     *reinterpret_cast<const uint32_t*>(q + 4));
    }
  }
};
