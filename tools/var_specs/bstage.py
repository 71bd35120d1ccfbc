# ADOPTED in round 4 (conv1.h stage_ld / stage_st); kept as the record of the A/B edit.
# fp32 backward, group B: the next frame's staging loads (image bytes, dY2, mask) issued at the
# top of B's step, under its conv1 weight-gradient MFMAs, and stored to LDS after them, instead
# of loads immediately followed by their LDS stores after the weight gradient (1.3-2.7k clocks
# of load latency per step on the bottleneck group, ppstamps32 r04f).
F = "conv1.h"
ANCHOR = "  if (is_a && nF > 0 && load_w2) c12_load_w2(w2t, wb, wave, lane);"
NEW_LAMBDAS = r'''  struct StRegs {
    uint4 nv[3];
    f32x4 nd2[ND2];
    uint32_t nmk;
  };
  auto stage_ld = [&](int fi, int fd, StRegs& r) {
    r.nmk = 0;
    if (fi >= 0) c1_load_frame<float>(x + (size_t)fi * IMG, tid, r.nv);
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
'''
VARIANTS = {
    "bstage": [
        (F, ANCHOR, NEW_LAMBDAS + ANCHOR),
        (F, "    for (int it = 1; it <= nF; ++it) {\n      // ---- conv1 weight gradient of frame it - 1",
            "    for (int it = 1; it <= nF; ++it) {\n      StRegs sr;\n      stage_ld(it < nF ? f0 + it : -1, it + 1 < nF ? f0 + it + 1 : -1, sr);\n      // ---- conv1 weight gradient of frame it - 1"),
        (F, "      stage(it < nF ? f0 + it : -1, it & 1, it + 1 < nF ? f0 + it + 1 : -1, (it + 1) & 1);\n      __syncthreads();",
            "      stage_st(it < nF ? f0 + it : -1, it & 1, it + 1 < nF ? f0 + it + 1 : -1, (it + 1) & 1, sr);\n      __syncthreads();"),
    ],
}
