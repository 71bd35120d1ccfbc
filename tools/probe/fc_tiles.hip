// Probe: the fp32 FC forward (Linear 1024 -> 256 + GELU at N = 1280) in the library's KW tile
// GEMM (gemm_tile<float, BR, BC, 128, 2, 4, FcFwd<float>, PF 2, KACC 1, KW>: 8 waves split each
// K chunk's k-steps) over several BR x BC tile shapes, 300 launches each, outputs compared
// bitwise with the library's 16 x 80 shape (the KW sum order does not depend on the tile).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I impala_amd/csrc tools/probe/fc_tiles.hip -o tools/probe/fc_tiles
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "ops.h"

#define CKH(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

template <int BR, int BC>
static void run(const FcFwd<float>& op, int N, int reps, float* dh, std::vector<float>& ref, bool first) {
  auto k = gemm_tile<float, BR, BC, 128, 2, 4, FcFwd<float>, 2, 1, true>;
  const long tiles = (long)((N + BC - 1) / BC) * (HID / BR);
  const int grid = (int)(tiles < 768 ? tiles : 768);
  for (int i = 0; i < 20; ++i) k<<<grid, 512>>>(op, HID / BR);
  CKH(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CKH(hipEventCreate(&e0)); CKH(hipEventCreate(&e1));
  CKH(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) k<<<grid, 512>>>(op, HID / BR);
  CKH(hipEventRecord(e1));
  CKH(hipEventSynchronize(e1));
  float ms; CKH(hipEventElapsedTime(&ms, e0, e1));
  std::vector<float> out((size_t)N * HID);
  CKH(hipMemcpy(out.data(), dh, out.size() * 4, hipMemcpyDeviceToHost));
  if (first) ref = out;
  const bool same = std::memcmp(out.data(), ref.data(), out.size() * 4) == 0;
  std::printf("%3d x %3d  %4ld tiles  %8.2f us  %s\n", BR, BC, tiles, ms * 1e3f / reps,
              same ? "bitwise = 16x80" : "DIFFERENT");
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 1280;
  std::vector<float> w((size_t)HID * FLAT), y((size_t)N * YLD), b(HID);
  uint64_t s = 777;
  auto rnd = [&]() { s = s * 6364136223846793005ULL + 1442695040888963407ULL; return ((s >> 11) * (1.0 / 9007199254740992.0)) * 2 - 1; };
  for (auto& v : w) v = (float)(rnd() * 0.05);
  for (auto& v : y) v = (float)(rnd() * 2.0);
  for (auto& v : b) v = (float)(rnd() * 0.1);
  float *dw, *dy, *db, *dzg, *dh;
  CKH(hipMalloc(&dw, w.size() * 4)); CKH(hipMalloc(&dy, y.size() * 4)); CKH(hipMalloc(&db, HID * 4));
  CKH(hipMalloc(&dzg, (size_t)N * HID * 4)); CKH(hipMalloc(&dh, (size_t)N * HID * 4));
  CKH(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  CKH(hipMemcpy(dy, y.data(), y.size() * 4, hipMemcpyHostToDevice));
  CKH(hipMemcpy(db, b.data(), HID * 4, hipMemcpyHostToDevice));
  FcFwd<float> op{N, dw, db, dy, dzg, dh};
  std::vector<float> ref;
  const int reps = 300;
  run<16, 80>(op, N, reps, dh, ref, true);
  run<32, 48>(op, N, reps, dh, ref, false);
  run<16, 64>(op, N, reps, dh, ref, false);
  run<32, 32>(op, N, reps, dh, ref, false);
  run<16, 96>(op, N, reps, dh, ref, false);
  run<64, 32>(op, N, reps, dh, ref, false);
  run<32, 64>(op, N, reps, dh, ref, false);
  run<16, 80>(op, N, reps, dh, ref, false);
  return 0;
}
