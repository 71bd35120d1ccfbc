// LayerNorm backward + conv3 ReLU mask + conv3 input gradient + conv2 ReLU mask, fused per
// frame (the backward of models/models.py:66 LayerNorm and models/common.py:117-118 conv3).
//
//   dact3 = relu'(act3) * LN_bwd(dy)                  (dy from the FC dgrad, fp32)
//   dact2[iy][ix][ci] = relu'(act2) * sum_{kh,kw,oc} dact3[iy-kh][ix-kw][oc] W3[oc][kh][kw][ci]
//
// One frame per 4-wave group at a time, G groups per workgroup on alternating frames:
//   LN: wave w owns features 256 w .. 256 w + 255 (lane: 4 consecutive), the two per-frame
//       sums are combined through LDS; dact3 goes to HBM (for the conv3 weight gradient) and
//       to LDS
//   dgrad in scatter form: Z[p][tap][ci] = sum_oc dact3[p][oc] W3[oc][tap][ci] for the 16
//       conv3 output pixels p (one MFMA row tile; wave w owns ci tile w of every tap, its W3
//       fragments -- read k-major through the LDS transpose read -- in registers; K = 64),
//       then each input pixel gathers its <= 9 (p, tap) contributions from the fp32 Z in LDS
//       in a fixed order.  72 MFMAs per frame instead of the 216 of the gather form, and no
//       shifted-window LDS reads.
// LN gamma / beta gradient partials are kept per lane and written as one fp32 slab per
// workgroup (fixed-order combine of the groups), reduced by reduce_grads like the others.
#pragma once
#include "conv1.h"
#include "gemm.h"
#include "net.h"

using namespace net;

namespace lc3 {
constexpr int ZR = 9 * OC2 + 4;  // Z row (fp32): [tap][ci] of one output pixel, padded
}

template <typename T> constexpr int lnc3_groups() { return sizeof(T) == 2 ? 2 : 1; }
// threads of a launch: bf16 2 groups of 4 waves on alternating frames; fp32 8 waves on one
// frame (lnc3_body_f32)
template <typename T> constexpr int lnc3_threads() { return sizeof(T) == 2 ? 256 * lnc3_groups<T>() : 512; }

// fp32 LDS (bytes): Z (fp32 [16 + 1][ZR], row 16 zero), the dact3 tile [16][LD3], the LN sums
struct Lnc3F32 {
  static constexpr int LD3 = OC3 + 8;
  static constexpr int D3 = (P3 + 1) * lc3::ZR * 4, RED = D3 + P3 * LD3 * 4, BYTES = RED + 4 * 2 * 4;
};

// LDS of the body (bytes): the W3 staging / per-group Z + dact3 tiles, then red and comb
template <typename T> struct Lnc3Lds {
  static constexpr int VEC = 16 / (int)sizeof(T), LD3 = OC3 + 2 * VEC, LW = K3 + 2 * VEC;
  static constexpr int G = lnc3_groups<T>();
  static constexpr int ZB = (P3 + 1) * lc3::ZR * 4, GB = ZB + P3 * LD3 * (int)sizeof(T);
  static constexpr bool REG = sizeof(T) == 2;
  // W3 staging (bf16; fp32 loads its fragments from the transposed copy)
  static constexpr int STG = REG ? OC3 * LW * (int)sizeof(T) : 0;
  static constexpr int SMEM = STG > G * GB ? STG : G * GB;
  static constexpr int RED = SMEM, COMB = RED + G * 4 * 2 * 4;
  static constexpr int BYTES = sizeof(T) == 4 ? Lnc3F32::BYTES : COMB + 2 * FLAT * 4;
};

// The kernel body, on workgroup `wg` (frames wg*fpw ..) with the LDS passed in
// (Lnc3Lds<T>::BYTES), so a launch can run it ahead of another per-frame body.
template <typename T>
DEV void lnc3_body_g(const float* __restrict__ dy, const T* __restrict__ act3,
                   const float* __restrict__ stats, const float* __restrict__ gam,
                   const T* __restrict__ w3, const T* __restrict__ w3t,
                   const T* __restrict__ act2, T* __restrict__ dact3,
                   T* __restrict__ dact2, float* __restrict__ slab, int N, int fpw, int wg,
                   char* __restrict__ lds) {
  using F = Frag<T>;
  typedef typename F::vec V;
  constexpr int KPL = F::KPL, KS = F::KSTEP;
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int LD3 = OC3 + 2 * VEC;                 // dact3 row (80 bf16: conflict-free b128 reads)
  constexpr int LW = K3 + 2 * VEC;                   // staged W3 row (bit-2/3 swapped rows)
  constexpr int NKS = K3 / KS;
  constexpr int NKO = OC3 / KS;                      // k-steps per tap (K = oc)
  constexpr int G = lnc3_groups<T>();
  // one group's LDS: Z (fp32 [16 + 1][ZR]: row 16 stays zero, read by the gather's
  // out-of-range taps) then the dact3 tile (T [16][LD3]), in bytes
  constexpr int ZB = Lnc3Lds<T>::ZB, GB = Lnc3Lds<T>::GB;
  constexpr bool REG = sizeof(T) == 2;               // bf16: W3 fragments in registers
  static_assert(GB % 16 == 0 && Lnc3Lds<T>::SMEM % 16 == 0, "group alignment");
  char* smem_b = lds;
  float (*red)[4][2] = reinterpret_cast<float (*)[4][2]>(lds + Lnc3Lds<T>::RED);
  float* comb = reinterpret_cast<float*>(lds + Lnc3Lds<T>::COMB);
  T* smem = reinterpret_cast<T*>(smem_b);
  const int grp = threadIdx.x >> 8, tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  float* zs = reinterpret_cast<float*>(smem_b + grp * GB);
  T* d3s = reinterpret_cast<T*>(smem_b + grp * GB + ZB);
  const int f0 = wg * fpw, f1 = min(N, f0 + fpw);
  const int kl = KPL * (lane >> 4);
  // this lane's LN features j = 256 w + 4 lane + q  (pixel p = j / 64, channel c = j % 64)
  const int j0 = 256 * wave + 4 * lane, p0 = j0 >> 6, c0 = j0 & 63;

  // ---- per-frame inputs, prefetched one frame ahead ----
  f32x4 ndy = f32x4{0.f, 0.f, 0.f, 0.f};
  float nx[4] = {0.f, 0.f, 0.f, 0.f}, nm = 0.f, nr = 0.f, na[3][4];
  auto fetch = [&](int f) {
    ndy = *reinterpret_cast<const f32x4*>(dy + (size_t)f * FLAT + j0);
    load4(act3 + (size_t)f * FLAT + j0, nx);
    nm = stats[2 * f];
    nr = stats[2 * f + 1];
#pragma unroll
    for (int r = 0; r < 3; ++r) {  // gather items e = tid + 256 r: pixel e / 16, channels 4 (e % 16)
      const int e = min(tid + 256 * r, P2 * 16 - 1);
      load4(act2 + ((size_t)f * P2 + (e >> 4)) * OC2 + 4 * (e & 15), na[r]);
    }
  };
  if (f0 + grp < f1) fetch(f0 + grp);
  float gm[4], dg[4] = {0.f, 0.f, 0.f, 0.f}, db[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 4; ++q) gm[q] = gam[j0 + q];

  // ---- W3 fragments: B[k = oc][n = ci] = W3[oc][tap][ci] of every tap (k-major), held in
  // registers for the whole frame run (bf16 72, fp32 144 VGPRs) ----
  V wa[NKS];
  if constexpr (!REG) {
    // fp32: 16-byte loads from the transposed copy w3t[tap*64 + ci][oc] (k = oc contiguous),
    // all 36 in flight at once, consumed in the frame loop
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int k = ks * KS, tap = k >> 6, oc0 = k & 63;
      wa[ks] = F::load(w3t + (size_t)(tap * OC2 + 16 * wave + (lane & 15)) * OC3 + oc0 + kl);
    }
  } else {
    constexpr int NV = OC3 * K3 / VEC, NT = 256 * G, NPT = (NV + NT - 1) / NT;
    V wv[NPT];  // all loads in flight at once, then the LDS stores
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = (int)threadIdx.x + i * NT;
      if (e < NV) wv[i] = *reinterpret_cast<const V*>(w3 + (size_t)e * VEC);
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = (int)threadIdx.x + i * NT;
      if (e < NV) {
        const int r = e / (K3 / VEC), c = (e % (K3 / VEC)) * VEC;
        *reinterpret_cast<V*>(smem + wg_row(r) * LW + c) = wv[i];
      }
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int k = ks * KS, tap = k >> 6, oc0 = k & 63;
      wa[ks] = lds_frag_k_sw(smem + oc0 * LW + tap * OC2 + 16 * wave, LW, lane);
    }
    __syncthreads();  // the staging area becomes the Z / dact3 tiles
  }
  // consume the prologue loads before the loop (see conv1.h: waits merged over the back-edge)
#pragma unroll
  for (int q = 0; q < 4; ++q) asm volatile("" ::"v"(gm[q]));

  for (int e = tid; e < lc3::ZR / 4; e += 256)  // the zero row of this group's Z tile
    *reinterpret_cast<f32x4*>(zs + P3 * lc3::ZR + 4 * e) = f32x4{0.f, 0.f, 0.f, 0.f};
  const int n_it = (f1 - f0 + G - 1) / G;
  for (int it = 0; it < n_it; ++it) {
    const int f = f0 + G * it + grp;
    const bool active = f < f1;
    __syncthreads();  // the previous frame's readers of the cell grid / red are done
    float d[4], x[4], xh[4], am[3][4];
    const float mean = nm, rstd = nr;
#pragma unroll
    for (int q = 0; q < 4; ++q) { d[q] = ndy[q]; x[q] = nx[q]; }
#pragma unroll
    for (int pt = 0; pt < 3; ++pt)
#pragma unroll
      for (int q = 0; q < 4; ++q) am[pt][q] = na[pt][q];
    // ---- LayerNorm backward: the two per-frame sums ----
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      xh[q] = (x[q] - mean) * rstd;
      const float gd = d[q] * gm[q];
      s1 += gd;
      s2 += gd * xh[q];
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) { red[grp][wave][0] = s1; red[grp][wave][1] = s2; }
    __syncthreads();
    if (f + G < f1) fetch(f + G);
    if (active) {
      const float S1 = (red[grp][0][0] + red[grp][1][0] + red[grp][2][0] + red[grp][3][0]) * (1.f / FLAT);
      const float S2 = (red[grp][0][1] + red[grp][1][1] + red[grp][2][1] + red[grp][3][1]) * (1.f / FLAT);
      float o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dg[q] += d[q] * xh[q];
        db[q] += d[q];
        const float gx = rstd * (d[q] * gm[q] - S1 - xh[q] * S2);
        o[q] = x[q] > 0.f ? gx : 0.f;
      }
      store4(dact3 + (size_t)f * FLAT + j0, o);
      store4(d3s + p0 * LD3 + c0, o);
    }
    __syncthreads();
    if (active) {
      // ---- Z[p][tap][ci] = sum_oc dact3[p][oc] W3[oc][tap][ci]: wave w, ci tile w ----
      V a[NKO];
#pragma unroll
      for (int ko = 0; ko < NKO; ++ko)
        a[ko] = *reinterpret_cast<const V*>(d3s + (lane & 15) * LD3 + ko * KS + kl);
      // the nine taps' accumulators side by side: MFMA e of every tap before e + 1 (F::mma_e).
      // Z^T tiles (A = the W3 fragments, rows = ci; B = the dact3 rows, cols = p): a lane holds
      // four consecutive channels of one pixel and stores them with one 16-byte write (the
      // products and their k order are those of Z = dact3 x W3)
      f32x4 acc[9];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) acc[tap] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ko = 0; ko < NKO; ++ko)
#pragma unroll
        for (int e = 0; e < F::NE; ++e)
#pragma unroll
          for (int tap = 0; tap < 9; ++tap) acc[tap] = F::mma_e(e, wa[tap * NKO + ko], a[ko], acc[tap]);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
        *reinterpret_cast<f32x4*>(zs + (lane & 15) * lc3::ZR + tap * OC2 + 16 * wave + 4 * (lane >> 4)) = acc[tap];
    }
    __syncthreads();
    if (active) {
      // ---- col2im gather in a fixed (kh, kw) order + conv2's ReLU mask -> dact2 ----
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int e = tid + 256 * r;
        if (e < P2 * 16) {
          const int px = e >> 4, ci = 4 * (e & 15), iy = px / H2, ix = px - iy * H2;
          // branch-free: out-of-range taps read the zero row (+ 0 leaves the sum unchanged)
          f32x4 zt[9];
#pragma unroll
          for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
              const int oy = iy - kh, ox = ix - kw;
              const bool ok = oy >= 0 && oy < H3 && ox >= 0 && ox < H3;
              zt[kh * 3 + kw] = *reinterpret_cast<const f32x4*>(
                  zs + (ok ? oy * H3 + ox : P3) * lc3::ZR + (kh * 3 + kw) * OC2 + ci);
            }
          f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int t = 0; t < 9; ++t) sum += zt[t];
          float o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = am[r][q] > 0.f ? sum[q] : 0.f;
          store4(dact2 + ((size_t)f * P2 + px) * OC2 + ci, o);
        }
      }
    }
  }
  // ---- gamma / beta partials: fixed-order combine of the groups -> slab [2][1024] ----
  __syncthreads();
  if (grp == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) { comb[j0 + q] = dg[q]; comb[FLAT + j0 + q] = db[q]; }
  }
  for (int g = 1; g < G; ++g) {
    __syncthreads();
    if (grp == g) {
#pragma unroll
      for (int q = 0; q < 4; ++q) { comb[j0 + q] += dg[q]; comb[FLAT + j0 + q] += db[q]; }
    }
  }
  __syncthreads();
  for (int e = (int)threadIdx.x; e < 2 * FLAT / 4; e += 256 * G)
    *reinterpret_cast<f32x4*>(slab + (size_t)wg * 2 * FLAT + 4 * e) =
        *reinterpret_cast<const f32x4*>(comb + 4 * e);
}

// fp32: one frame at a time on 8 waves (512 threads: the shape of the two-group conv12 body it
// is fused with, whose launch bounds leave 256 VGPRs per lane -- the one-group form held all
// nine taps' W3 fragments, 144 VGPRs, on every wave).  Two roles, each a separate code path
// (ROLE is a template parameter; a workgroup runs role 0 on waves 0..3 and role 1 on waves
// 4..7, with the same barriers):
//   role 0: the LayerNorm backward (lane: 4 consecutive features, as in the one-group form) and
//           half of the gather; its registers stay free for the conv12 body's W2 fragments,
//           which `pre(k)` loads during the frames, one tap (32 KB per workgroup) in frame
//           1 + k after that frame's prefetch, so the W3 burst is not delayed and no frame's
//           loads queue behind all 128 KB (one 128 KB burst in frame 1 made the LayerNorm part
//           8.4k clocks longer: the CU's load path, not the latency, bounds it);
//   role 1: the W3 fragments of all nine taps (ci tile = wave & 3), the scatter GEMM, the other
//           half of the gather.
// Same sums in the same order as the one-group form.
template <int ROLE, class Pre>
DEV void lnc3_body_f32r(const float* __restrict__ dy, const float* __restrict__ act3,
                        const float* __restrict__ stats, const float* __restrict__ gam,
                        const float* __restrict__ w3t, const float* __restrict__ act2,
                        float* __restrict__ dact3, float* __restrict__ dact2, float* __restrict__ slab,
                        int N, int fpw, int wg, char* __restrict__ lds, Pre&& pre) {
  using F = Frag<float>;
  typedef F::vec V;
  constexpr int KS = F::KSTEP, NKO = OC3 / KS, LD3 = Lnc3F32::LD3;
  constexpr int NGI = (P2 * 16 + 511) / 512;  // gather items per thread
  constexpr bool LN = ROLE == 0;
  float* zs = reinterpret_cast<float*>(lds);
  float* d3s = reinterpret_cast<float*>(lds + Lnc3F32::D3);
  float (*red)[2] = reinterpret_cast<float (*)[2]>(lds + Lnc3F32::RED);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int f0 = wg * fpw, f1 = min(N, f0 + fpw);
  const int kl = 4 * (lane >> 4);
  const int j0 = 256 * (wave & 3) + 4 * lane, p0 = j0 >> 6, c0 = j0 & 63;
  const int ct = wave & 3;  // Z: ci tile
  f32x4 ndy = f32x4{0.f, 0.f, 0.f, 0.f};
  float nx[4] = {0.f, 0.f, 0.f, 0.f}, nm = 0.f, nr = 0.f, na[NGI][4];
  auto fetch = [&](int f) {
    if constexpr (LN) {
      ndy = *reinterpret_cast<const f32x4*>(dy + (size_t)f * FLAT + j0);
      load4(act3 + (size_t)f * FLAT + j0, nx);
      nm = stats[2 * f];
      nr = stats[2 * f + 1];
    }
#pragma unroll
    for (int r = 0; r < NGI; ++r) {  // gather items e = t + 512 r: pixel e / 16, channels 4 (e % 16)
      const int e = min(t + 512 * r, P2 * 16 - 1);
      load4(act2 + ((size_t)f * P2 + (e >> 4)) * OC2 + 4 * (e & 15), na[r]);
    }
  };
  if (f0 < f1) fetch(f0);
  float gm[4], dg[4] = {0.f, 0.f, 0.f, 0.f}, db[4] = {0.f, 0.f, 0.f, 0.f};
  // W3 fragments of the nine taps (role 1), from the transposed copy w3t[tap*64 + ci][oc]
  V wa[LN ? 1 : 9][NKO];
  if constexpr (LN) {
#pragma unroll
    for (int q = 0; q < 4; ++q) gm[q] = gam[j0 + q];
#pragma unroll
    for (int q = 0; q < 4; ++q) asm volatile("" ::"v"(gm[q]));
  } else {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int ko = 0; ko < NKO; ++ko)
        wa[tap][ko] = F::load(w3t + (size_t)(tap * OC2 + 16 * ct + (lane & 15)) * OC3 + ko * KS + kl);
  }
  for (int e = t; e < lc3::ZR / 4; e += 512)  // the Z tile's zero row
    *reinterpret_cast<f32x4*>(zs + P3 * lc3::ZR + 4 * e) = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int f = f0; f < f1; ++f) {
    __syncthreads();  // the previous frame's readers of Z / dact3 / red are done
    float am[NGI][4];
#pragma unroll
    for (int r = 0; r < NGI; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) am[r][q] = na[r][q];
    // ---- LayerNorm backward (role 0): the two per-frame sums, then dact3 ----
    float d[4], x[4], xh[4];
    const float mean = nm, rstd = nr;
    if constexpr (LN) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d[q] = ndy[q];
        x[q] = nx[q];
        xh[q] = (x[q] - mean) * rstd;
        const float gd = d[q] * gm[q];
        s1 += gd;
        s2 += gd * xh[q];
      }
      s1 = wave_sum(s1);
      s2 = wave_sum(s2);
      if (lane == 0) { red[wave][0] = s1; red[wave][1] = s2; }
    }
    __syncthreads();
    if (f + 1 < f1) fetch(f + 1);
    if constexpr (LN) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (f == f0 + 1 + k) pre(k);
      const float S1 = (red[0][0] + red[1][0] + red[2][0] + red[3][0]) * (1.f / FLAT);
      const float S2 = (red[0][1] + red[1][1] + red[2][1] + red[3][1]) * (1.f / FLAT);
      float o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dg[q] += d[q] * xh[q];
        db[q] += d[q];
        const float gx = rstd * (d[q] * gm[q] - S1 - xh[q] * S2);
        o[q] = x[q] > 0.f ? gx : 0.f;
      }
      store4(dact3 + (size_t)f * FLAT + j0, o);
      store4(d3s + p0 * LD3 + c0, o);
    }
    __syncthreads();
    // ---- Z[p][tap][ci] = sum_oc dact3[p][oc] W3[oc][tap][ci] (role 1): Z^T tiles, the nine
    // taps' accumulators side by side (MFMA e of every tap before e + 1); a lane stores four
    // consecutive channels of one pixel per tap ----
    if constexpr (!LN) {
      V a[NKO];
#pragma unroll
      for (int ko = 0; ko < NKO; ++ko)
        a[ko] = *reinterpret_cast<const V*>(d3s + (lane & 15) * LD3 + ko * KS + kl);
      f32x4 acc[9];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) acc[tap] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ko = 0; ko < NKO; ++ko)
#pragma unroll
        for (int e = 0; e < F::NE; ++e)
#pragma unroll
          for (int tap = 0; tap < 9; ++tap) acc[tap] = F::mma_e(e, wa[tap][ko], a[ko], acc[tap]);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
        *reinterpret_cast<f32x4*>(zs + (lane & 15) * lc3::ZR + tap * OC2 + 16 * ct + kl) = acc[tap];
    }
    __syncthreads();
    // ---- col2im gather in a fixed (kh, kw) order + conv2's ReLU mask -> dact2 ----
#pragma unroll
    for (int r = 0; r < NGI; ++r) {
      const int e = t + 512 * r;
      if (e < P2 * 16) {
        const int px = e >> 4, ci = 4 * (e & 15), iy = px / H2, ix = px - iy * H2;
        f32x4 zt[9];
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int oy = iy - kh, ox = ix - kw;
            const bool ok = oy >= 0 && oy < H3 && ox >= 0 && ox < H3;
            zt[kh * 3 + kw] = *reinterpret_cast<const f32x4*>(
                zs + (ok ? oy * H3 + ox : P3) * lc3::ZR + (kh * 3 + kw) * OC2 + ci);
          }
        f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 9; ++k) sum += zt[k];
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = am[r][q] > 0.f ? sum[q] : 0.f;
        store4(dact2 + ((size_t)f * P2 + px) * OC2 + ci, o);
      }
    }
  }
  if constexpr (LN) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (f1 - f0 < k + 2) pre(k);
    // ---- gamma / beta partials -> slab [2][1024] ----
    *reinterpret_cast<f32x4*>(slab + (size_t)wg * 2 * FLAT + j0) = f32x4{dg[0], dg[1], dg[2], dg[3]};
    *reinterpret_cast<f32x4*>(slab + (size_t)wg * 2 * FLAT + FLAT + j0) = f32x4{db[0], db[1], db[2], db[3]};
  }
}

template <typename T>
DEV void lnc3_body(const float* __restrict__ dy, const T* __restrict__ act3,
                   const float* __restrict__ stats, const float* __restrict__ gam,
                   const T* __restrict__ w3, const T* __restrict__ w3t,
                   const T* __restrict__ act2, T* __restrict__ dact3,
                   T* __restrict__ dact2, float* __restrict__ slab, int N, int fpw, int wg,
                   char* __restrict__ lds) {
  if constexpr (sizeof(T) == 4) {
    if (threadIdx.x < 256)
      lnc3_body_f32r<0>(dy, act3, stats, gam, w3t, act2, dact3, dact2, slab, N, fpw, wg, lds, [](int) {});
    else
      lnc3_body_f32r<1>(dy, act3, stats, gam, w3t, act2, dact3, dact2, slab, N, fpw, wg, lds, [](int) {});
  } else
    lnc3_body_g<T>(dy, act3, stats, gam, w3, w3t, act2, dact3, dact2, slab, N, fpw, wg, lds);
}

template <typename T>
__global__ __launch_bounds__(lnc3_threads<T>()) void lnc3_bwd(
    const float* __restrict__ dy, const T* __restrict__ act3, const float* __restrict__ stats,
    const float* __restrict__ gam, const T* __restrict__ w3, const T* __restrict__ w3t,
    const T* __restrict__ act2, T* __restrict__ dact3, T* __restrict__ dact2,
    float* __restrict__ slab, int N, int fpw) {
  __shared__ __attribute__((aligned(16))) char lds[Lnc3Lds<T>::BYTES];
  lnc3_body<T>(dy, act3, stats, gam, w3, w3t, act2, dact3, dact2, slab, N, fpw, (int)blockIdx.x, lds);
}

// LayerNorm backward + conv3 input gradient, then conv2 input gradient + conv1 weight gradient,
// in ONE launch: both are per-frame chains over the same run of frames per workgroup, so the
// workgroup runs lnc3_body on its frames, then conv12_bwd_body on the same frames (dact2 comes
// back from the workgroup's own global stores, ordered by the barrier between the bodies).
// The two bodies share the LDS (its size is the larger of theirs).  The conv3 / conv2 weight
// gradients, which need dact3 / dact2 of all frames, run after it.
template <typename T, class O = ObsDirect>
__global__ __launch_bounds__(lnc3_threads<T>()) void lnc3_conv12_bwd(
    const float* __restrict__ dy, const T* __restrict__ act3, const float* __restrict__ stats,
    const float* __restrict__ gam, const T* __restrict__ w3, const T* __restrict__ w3t,
    const T* __restrict__ act2, T* __restrict__ dact3, T* __restrict__ dact2,
    float* __restrict__ ln_slab, const uint8_t* __restrict__ x, const T* __restrict__ w2,
    const T* __restrict__ w2t, const uint32_t* __restrict__ mask1,
    float* __restrict__ c1_slab, float* __restrict__ c1_slab_bias, int N, int fpw, const O rm) {
  static_assert(lnc3_threads<T>() == 256 * c12_groups<T>(), "one block shape for both bodies");
  constexpr int B1 = Lnc3Lds<T>::BYTES, B2 = C12BLds<T>::BYTES;
  __shared__ __attribute__((aligned(16))) char lds[B1 > B2 ? B1 : B2];
  if constexpr (sizeof(T) == 4) {
    // fp32: each 4-wave group runs its role of both bodies as one code path, so group A's W2
    // fragments (loaded during the LayerNorm frames) and group B's W3 fragments / weight-gradient
    // accumulators never share the register budget
    const float* w3f = reinterpret_cast<const float*>(w3t);
    const float* w2f = reinterpret_cast<const float*>(w2t);
    const float* a3 = reinterpret_cast<const float*>(act3);
    const float* a2 = reinterpret_cast<const float*>(act2);
    float* d3 = reinterpret_cast<float*>(dact3);
    float* d2 = reinterpret_cast<float*>(dact2);
    Frag<float>::vec wb[4][OC2 / Frag<float>::KSTEP][2];
    const int wg = (int)blockIdx.x;
    if (threadIdx.x < 256) {
      const int cls = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
      lnc3_body_f32r<0>(dy, a3, stats, gam, w3f, a2, d3, d2, ln_slab, N, fpw, wg, lds,
                        [&](int k) { c12_load_w2(w2f, wb, cls, lane, k, k + 1); });
      __syncthreads();  // this workgroup's dact2 stores are visible to all its waves; LDS is reused
      conv12_bwd_body_f32<0, O>(x, w2f, d2, mask1, c1_slab, c1_slab_bias, N, fpw, wg, lds, wb, false, rm);
    } else {
      lnc3_body_f32r<1>(dy, a3, stats, gam, w3f, a2, d3, d2, ln_slab, N, fpw, wg, lds, [](int) {});
      __syncthreads();
      conv12_bwd_body_f32<1, O>(x, w2f, d2, mask1, c1_slab, c1_slab_bias, N, fpw, wg, lds, wb, false, rm);
    }
  } else {
    lnc3_body<T>(dy, act3, stats, gam, w3, w3t, act2, dact3, dact2, ln_slab, N, fpw, (int)blockIdx.x, lds);
    __syncthreads();  // this workgroup's dact2 stores are visible to all its waves; LDS is reused
    conv12_bwd_body<T, O>(x, w2, w2t, dact2, mask1, c1_slab, c1_slab_bias, N, fpw, (int)blockIdx.x, lds, rm);
  }
}
