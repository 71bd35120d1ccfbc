// Probe: the fp32 FC forward (Linear 1024 -> 256 + GELU at N = 1280) as the library runs it
// (gemm_tile<float> KW, impala.hip FCF_*) against the same GEMM on split bf16 planes
// (gemm_tile NP = 3, 9 plane products on the bf16 MFMA) and plain bf16.  Times each over 200
// launches with events and checks h against an fp64 host reference.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I impala_amd/csrc tools/probe/fc_split.hip -o tools/probe/fc_split
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "ops.h"

// The fp32 FC forward on split planes (probe only: measured slower, see the header) (gemm_tile NP = 3, gemm.h): Wfc and y each as three bf16
// planes (hi, mid, lo; plane p at p * a_ps / p * y_ps elements from plane 0), every plane
// product on the bf16 MFMA, accumulated in fp32; bias + GELU epilogue as FcFwd<float>.
struct FcFwdP {
  static constexpr bool A_KMAJOR = false;
  static constexpr bool TILE_EPI = false;
  static constexpr int K = FLAT;
  int C;
  const __bf16* w;
  int a_ps;
  const float* b;
  const __bf16* y;
  int y_ps;
  float* zg;
  float* h;
  struct ColCtx { const __bf16* p; };
  DEV ColCtx col_ctx(int c) const { return ColCtx{y + (size_t)c * YLD}; }
  DEV const __bf16* a_row(int r, int) const { return w + r * K; }
  DEV Frag<__bf16>::vec load_b(const ColCtx& cc, int k, int p) const {
    return Frag<__bf16>::load(cc.p + k + (size_t)p * y_ps);
  }
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


#define CKH(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

static uint16_t bf16_rne(float x) {
  uint32_t u; std::memcpy(&u, &x, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf16_f(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; std::memcpy(&f, &u, 4); return f; }
static void split3h(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = bf16_rne(x);
  const float r1 = x - bf16_f(h);
  m = bf16_rne(r1);
  l = bf16_rne(r1 - bf16_f(m));
}

template <class K, class... A>
static float time_us(K kern, dim3 g, dim3 b, int reps, A... args) {
  hipEvent_t e0, e1;
  CKH(hipEventCreate(&e0)); CKH(hipEventCreate(&e1));
  for (int i = 0; i < 10; ++i) kern<<<g, b>>>(args...);
  CKH(hipDeviceSynchronize());
  CKH(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) kern<<<g, b>>>(args...);
  CKH(hipEventRecord(e1));
  CKH(hipEventSynchronize(e1));
  float ms; CKH(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 1280;
  const int reps = 200;
  std::vector<float> w((size_t)HID * FLAT), y((size_t)N * YLD), b(HID);
  uint64_t s = 12345;
  auto rnd = [&]() { s = s * 6364136223846793005ULL + 1442695040888963407ULL; return ((s >> 11) * (1.0 / 9007199254740992.0)) * 2 - 1; };
  for (auto& v : w) v = (float)(rnd() * 0.05);
  for (auto& v : y) v = (float)(rnd() * 2.0);
  for (auto& v : b) v = (float)(rnd() * 0.1);
  // host planes
  std::vector<uint16_t> w3(3 * w.size()), y3(3 * y.size()), wb(w.size()), yb(y.size());
  for (size_t i = 0; i < w.size(); ++i) { split3h(w[i], w3[i], w3[w.size() + i], w3[2 * w.size() + i]); wb[i] = w3[i]; }
  for (size_t i = 0; i < y.size(); ++i) { split3h(y[i], y3[i], y3[y.size() + i], y3[2 * y.size() + i]); yb[i] = y3[i]; }
  // fp64 reference of h = gelu(W y + b)
  std::vector<double> href((size_t)N * HID);
  for (int n = 0; n < N; ++n)
    for (int o = 0; o < HID; ++o) {
      double acc = b[o];
      for (int k = 0; k < FLAT; ++k) acc += (double)w[(size_t)o * FLAT + k] * y[(size_t)n * YLD + k];
      href[(size_t)n * HID + o] = 0.5 * acc * (1.0 + std::erf(acc / std::sqrt(2.0)));
    }
  float *dw, *dy, *db, *dzg, *dh;
  __bf16 *dw3, *dy3, *dwb, *dyb, *dhb;
  CKH(hipMalloc(&dw, w.size() * 4)); CKH(hipMalloc(&dy, y.size() * 4)); CKH(hipMalloc(&db, HID * 4));
  CKH(hipMalloc(&dzg, (size_t)N * HID * 4)); CKH(hipMalloc(&dh, (size_t)N * HID * 4));
  CKH(hipMalloc(&dw3, w3.size() * 2)); CKH(hipMalloc(&dy3, y3.size() * 2));
  CKH(hipMalloc(&dwb, wb.size() * 2)); CKH(hipMalloc(&dyb, yb.size() * 2)); CKH(hipMalloc(&dhb, (size_t)N * HID * 2));
  CKH(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  CKH(hipMemcpy(dy, y.data(), y.size() * 4, hipMemcpyHostToDevice));
  CKH(hipMemcpy(db, b.data(), HID * 4, hipMemcpyHostToDevice));
  CKH(hipMemcpy(dw3, w3.data(), w3.size() * 2, hipMemcpyHostToDevice));
  CKH(hipMemcpy(dy3, y3.data(), y3.size() * 2, hipMemcpyHostToDevice));
  CKH(hipMemcpy(dwb, wb.data(), wb.size() * 2, hipMemcpyHostToDevice));
  CKH(hipMemcpy(dyb, yb.data(), yb.size() * 2, hipMemcpyHostToDevice));
  int ncu = 256;
  auto pgrid = [&](long tiles) { return (int)std::min<long>(tiles, 3L * ncu); };
  std::vector<float> out((size_t)N * HID);
  auto check = [&](const char* name, float us) {
    CKH(hipMemcpy(out.data(), dh, out.size() * 4, hipMemcpyDeviceToHost));
    double md = 0, mr = 0, num = 0, den = 0;
    for (size_t i = 0; i < out.size(); ++i) {
      const double d = std::fabs(out[i] - href[i]);
      md = std::max(md, d);
      num += d * d; den += href[i] * href[i];
    }
    std::printf("%-28s %8.2f us   max|d| %.3e  rel-L2 %.3e\n", name, us, md, std::sqrt(num / den));
  };
  {  // library fp32 config: gemm_tile<float, 16, 80, 128, 2, 4, FcFwd<float>, 2, 1, KW>
    FcFwd<float> op{N, dw, db, dy, dzg, dh};
    auto k = gemm_tile<float, 16, 80, 128, 2, 4, FcFwd<float>, 2, 1, true>;
    const float us = time_us(k, dim3(pgrid((long)((N + 79) / 80) * (HID / 16))), dim3(512), reps, op, HID / 16);
    check("fp32 f32-MFMA (library)", us);
  }
#define SPLIT_CASE(BR, BC, BK, WR, WC)                                                                  \
  {                                                                                                    \
    FcFwdP op{N, dw3, HID * FLAT, db, dy3, N * YLD, dzg, dh};                                          \
    auto k = gemm_tile<__bf16, BR, BC, BK, WR, WC, FcFwdP, 1, 1, false, 3>;                            \
    const float us = time_us(k, dim3(pgrid((long)((N + BC - 1) / BC) * (HID / BR))), dim3(64 * WR * WC), reps, op, HID / BR); \
    check("split3x9 " #BR "x" #BC " bk" #BK " " #WR "x" #WC, us);                                      \
  }
  SPLIT_CASE(32, 32, 64, 2, 2)
  SPLIT_CASE(32, 32, 128, 2, 2)
  SPLIT_CASE(64, 32, 64, 2, 2)
  SPLIT_CASE(32, 64, 64, 2, 2)
  SPLIT_CASE(64, 64, 64, 2, 2)
  {  // plain bf16 (the bf16 mode's config), output to bf16 h: timing only
    FcFwd<__bf16> op{N, dwb, db, dyb, dzg, dhb};
    auto k = gemm_tile<__bf16, 32, 32, 256, 2, 2, FcFwd<__bf16>>;
    const float us = time_us(k, dim3(pgrid((long)((N + 31) / 32) * (HID / 32))), dim3(256), reps, op, HID / 32);
    std::printf("%-28s %8.2f us   (timing only)\n", "bf16 (bf16 mode)", us);
  }
  return 0;
}
