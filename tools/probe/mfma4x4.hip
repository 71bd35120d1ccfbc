// Layout probe of v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4x4x1, f32): lane l supplies a = A_l,
// b = B_l; prints every lane's 4 result registers so the A / B / D lane maps can be read off.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void probe(float* out, int mode) {
  const int l = threadIdx.x;
  // mode 0: a = 1 on lane l0 only (l0 = 5), b = lane id + 1  -> which outputs see lane 5's A
  // mode 1: a = lane id + 1, b = 1 on lane 5 only           -> which outputs see lane 5's B
  const float a = mode == 0 ? (l == 5 ? 1.f : 0.f) : (float)(l + 1);
  const float b = mode == 0 ? (float)(l + 1) : (l == 5 ? 1.f : 0.f);
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}
// issue rate: 256 rounds of 4 independent accumulators, one wave per SIMD (4 waves)
template <int KIND>
__global__ void rate(float* out, long long* cyc) {
  const int l = threadIdx.x & 63;
  float a = (float)l * 1e-3f, b = 1.f - (float)l * 1e-3f;
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
  for (int i = 0; i < 256; ++i) {
    if (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
    } else {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
  }
  const f32x4 s = c0 + c1 + c2 + c3;
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = s[0] + s[1] + s[2] + s[3];
  if (l == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 4 * 4);
  float h[256];
  for (int mode = 0; mode < 2; ++mode) {
    probe<<<1, 64>>>(d, mode);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("mode %d (nonzero outputs: lane.reg=value)\n", mode);
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r)
        if (h[l * 4 + r] != 0.f) printf(" %d.%d=%g", l, r, h[l * 4 + r]);
    printf("\n");
  }
  long long* dc;
  hipMalloc(&dc, 4 * sizeof(long long));
  long long hc[4];
  rate<0><<<1, 256>>>(d, dc);
  rate<0><<<1, 256>>>(d, dc);
  hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
  printf("4x4x1_16b f32: 1024 MFMAs per wave: %lld %lld %lld %lld ticks (%.2f per MFMA)\n", hc[0], hc[1], hc[2], hc[3], hc[0] / 1024.0);
  rate<1><<<1, 256>>>(d, dc);
  rate<1><<<1, 256>>>(d, dc);
  hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
  printf("16x16x4 f32: 1024 MFMAs per wave: %lld %lld %lld %lld ticks (%.2f per MFMA)\n", hc[0], hc[1], hc[2], hc[3], hc[0] / 1024.0);
  return 0;
}
