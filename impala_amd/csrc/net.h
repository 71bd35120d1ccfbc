// Geometry of the reference actor-critic (models/models.py:61-76, models/common.py:108-126)
// and the HBM layout of the kernel-side ("shadow") weights.
//
// Canonical parameters (the caller's flat fp32 buffer) are in torch state_dict order
// (SURVEY.md §8(a) a6).  The kernels never read them: the Adam kernel (and pack_params at
// bind time) re-emits every weight in the layout and dtype each GEMM consumes:
//
//   w1  [32][192]        k' = tap*48 + ci*16 + (kh%4)*4 + kw%4, tap = (kh/4)*2 + kw/4 (s2d)
//   w2  [64][512]        k = (kh*4+kw)*32 + ci                       (conv2, channels-last)
//   w3  [64][576]        k = (kh*3+kw)*64 + ci                       (conv3)
//   wfc [256][1024]      k = p*64 + c   (canonical column j = c*16 + p, NCHW flatten)
//   wh  [16][256]        rows 0..A-1 actor, row 15 critic, rest 0
// (the dgrads read w2 / w3 / wfc k-major through LDS: no transposed copies)
//   wht [256][32]        [j][o'], o' >= 16 zero
//   w2t [512][64]        [(kh*4+kw)*32 + ci][oc]   (fp32 only: the dgrads' B fragments as one
//   w3t [576][64]        [(kh*3+kw)*64 + ci][oc]    16-byte load, k = oc contiguous)
//   f32: b1[32] b2[64] b3[64] lng[1024] lnb[1024] (p*64+c order) bfc[256] bh[16]
#pragma once
#include <stddef.h>

namespace net {
constexpr int C0 = 3, H0 = 64, IMG = C0 * H0 * H0;        // 12288 bytes per frame
constexpr int OC1 = 32, KS1 = 8, ST1 = 4, H1 = 15, K1 = C0 * KS1 * KS1;    // 192
constexpr int OC2 = 64, KS2 = 4, ST2 = 2, H2 = 6, K2 = OC1 * KS2 * KS2;    // 512
constexpr int OC3 = 64, KS3 = 3, ST3 = 1, H3 = 4, K3 = OC2 * KS3 * KS3;    // 576
constexpr int P1 = H1 * H1, P2 = H2 * H2, P3 = H3 * H3;                   // 225, 36, 16
constexpr int FLAT = OC3 * P3;                                             // 1024
constexpr int HID = 256;
// row stride (elements) of the LayerNorm output y [N][YLD], the FC layer's input: a padded
// stride moves the rows of one 16-row fragment load off a common 4 KB alignment
constexpr int YLD = FLAT;
constexpr int HEADS = 16;     // actor rows 0..A-1, critic row 15
constexpr int HPAD = 32;      // padded K of the heads dgrad GEMM
constexpr int VCOL = 15;      // value column in the heads output
constexpr int MAX_A = 15;
constexpr float LN_EPS = 1e-5f;

// canonical flat-parameter segment offsets (A = number of actions)
struct Canon {
  size_t w1, b1, w2, b2, w3, b3, lng, lnb, wfc, bfc, wa, ba, wc, bc, total;
};
inline Canon canon(int A) {
  Canon c;
  size_t o = 0;
  c.w1 = o; o += (size_t)OC1 * K1;
  c.b1 = o; o += OC1;
  c.w2 = o; o += (size_t)OC2 * K2;
  c.b2 = o; o += OC2;
  c.w3 = o; o += (size_t)OC3 * K3;
  c.b3 = o; o += OC3;
  c.lng = o; o += FLAT;
  c.lnb = o; o += FLAT;
  c.wfc = o; o += (size_t)HID * FLAT;
  c.bfc = o; o += HID;
  c.wa = o; o += (size_t)A * HID;
  c.ba = o; o += A;
  c.wc = o; o += HID;
  c.bc = o; o += 1;
  c.total = o;
  return c;
}

// shadow-weight element offsets (elements of the compute type T), 64-element aligned
struct Shadow {
  size_t w1, w2, w3, wfc, wh, wht, w2t, w3t, total;
};
constexpr size_t al64(size_t x) { return (x + 63) & ~(size_t)63; }
inline Shadow shadow() {
  Shadow s;
  size_t o = 0;
  s.w1 = o; o = al64(o + (size_t)OC1 * K1);
  s.w2 = o; o = al64(o + (size_t)OC2 * K2);
  s.w3 = o; o = al64(o + (size_t)OC3 * K3);
  s.wfc = o; o = al64(o + (size_t)HID * FLAT);
  s.wh = o; o = al64(o + (size_t)HEADS * HID);
  s.wht = o; o = al64(o + (size_t)HID * HPAD);
  s.w2t = o; o = al64(o + (size_t)OC2 * K2);
  s.w3t = o; o = al64(o + (size_t)OC3 * K3);
  s.total = o;
  return s;
}
// fp32 side vector (biases, LayerNorm affine) offsets
struct Vecs {
  static constexpr size_t b1 = 0, b2 = 64, b3 = 128, lng = 192, lnb = 192 + 1024,
                          bfc = 192 + 2048, bh = 192 + 2048 + 256, total = 192 + 2048 + 256 + 64;
};
}  // namespace net
