// Probe: does the row stride of the FC operand y [1280][stride] fp32 (4 KB rows at stride 1024)
// throttle the FC GEMMs' loads?  256 workgroups each stream their 80 rows x 1024 floats in the
// two access patterns the FC kernels use:
//   "frag"  lane l reads 16 B of row (l & 15) at k = 4 (l >> 4) + 16 kb   (16 rows per load)
//   "tile"  16 lanes read one row's 256 B contiguous                       (4 rows per load)
// and sum them (kept live through one store per thread).  Prints us per launch (median of 20).
// build: hipcc --offload-arch=gfx950 -O3 -o rowstride tools/probe/rowstride.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void stream_rows(const float* __restrict__ y, int stride,
                                                   float* __restrict__ out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x % 16 * 80;  // 16 frame blocks of 80 rows, 16 workgroups each
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (MODE == 0) {
    // wave w: k in [256 w, 256 w + 256), 5 row groups of 16, 16 k-blocks, 4 loads in flight
    const int k0 = wave * 256 + 4 * (lane >> 4);
#pragma unroll
    for (int cf = 0; cf < 5; ++cf) {
      const float* p = y + (size_t)(r0 + cf * 16 + (lane & 15)) * stride + k0;
#pragma unroll
      for (int kb = 0; kb < 16; ++kb) acc += *reinterpret_cast<const f32x4*>(p + kb * 16);
    }
  } else {
    // 80 rows x 1024 floats = 80 x 64 vectors of 16 B; thread t takes vectors t, t + 256, ...
#pragma unroll 4
    for (int e = tid; e < 80 * 64; e += 256) {
      const int r = e / 64, v = e % 64;
      acc += *reinterpret_cast<const f32x4*>(y + (size_t)(r0 + r) * stride + v * 16 + (blockIdx.x / 16) % 1);
    }
  }
  out[blockIdx.x * 256 + tid] = acc[0] + acc[1] + acc[2] + acc[3];
}

int main() {
  const int rows = 1280, maxs = 2048;
  float *y, *out;
  hipMalloc(&y, (size_t)rows * maxs * 4);
  hipMalloc(&out, 256 * 256 * 4);
  hipMemset(y, 0, (size_t)rows * maxs * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int mode = 0; mode < 2; ++mode)
    for (int stride : {1024, 1028, 1040, 1056, 1088, 1152, 2048}) {
      std::vector<float> t;
      for (int it = 0; it < 22; ++it) {
        hipEventRecord(a);
        if (mode == 0)
          stream_rows<0><<<256, 256>>>(y, stride, out);
        else
          stream_rows<1><<<256, 256>>>(y, stride, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (it >= 2) t.push_back(ms * 1e3f);
      }
      std::sort(t.begin(), t.end());
      const double bytes = 256.0 * 80 * 1024 * 4;
      printf("%s stride %4d floats: %7.2f us  (%.1f TB/s from L2/MALL)\n", mode ? "tile" : "frag",
             stride, t[t.size() / 2], bytes / (t[t.size() / 2] * 1e-6) / 1e12);
    }
  return 0;
}
