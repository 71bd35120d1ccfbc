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

// the conv1 weight-gradient pattern: 6 accumulators (2 A x 3 B fragments of 4 elements), MFMAs
// in (j, e, i) or (e, i, j) order, operands rotated every step (VGPR copies, no memory)
template <int ORDER>
__global__ void rate6(float* out, long long* cyc) {
  const int l = threadIdx.x & 63;
  f32x4 fa[2][2], fb[2][3];
  for (int s = 0; s < 2; ++s) {
    for (int i = 0; i < 2; ++i) fa[s][i] = f32x4{l * 1e-3f + i, 1.f, 2.f, 3.f};
    for (int j = 0; j < 3; ++j) fb[s][j] = f32x4{l * 1e-3f - j, 1.f, 0.5f, 0.25f};
  }
  f32x4 acc[2][3];
  for (int i = 0; i < 2; ++i) for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_sched_barrier(0);
  const long long t0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  for (int st = 0; st < 64; ++st) {
    const int b = st & 1;
    if (ORDER == 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < 2; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[b][i][e], fb[b][j][e], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[b][i][e], fb[b][j][e], acc[i][j], 0, 0, 0);
    }
    // opaque operands: the compiler can neither fold nor hoist the steps
    for (int i = 0; i < 2; ++i) asm volatile("" : "+v"(fa[b ^ 1][i]));
    for (int j = 0; j < 3; ++j) asm volatile("" : "+v"(fb[b ^ 1][j]));
  }
  __builtin_amdgcn_sched_barrier(0);
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 2; ++i) for (int j = 0; j < 3; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[threadIdx.x] = s;
  if (l == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

// the same with the kernel's auxiliary work per 24-MFMA step: 16 LDS reads and 12 conversions
__global__ void rate6aux(float* out, long long* cyc) {
  __shared__ uint8_t img[16384];
  const int l = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 16384; i += 256) img[i] = (uint8_t)(i * 7);
  __syncthreads();
  f32x4 fa[2] = {f32x4{l * 1e-3f, 1.f, 2.f, 3.f}, f32x4{l * 2e-3f, 1.f, 2.f, 3.f}};
  uint32_t raw[12];
  for (int q = 0; q < 12; ++q) raw[q] = q;
  f32x4 acc[2][3];
  for (int i = 0; i < 2; ++i) for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_sched_barrier(0);
  const long long t0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  for (int st = 0; st < 64; ++st) {
    f32x4 fb[3];
    for (int j = 0; j < 3; ++j) fb[j] = f32x4{(float)raw[4 * j], (float)raw[4 * j + 1], (float)raw[4 * j + 2], (float)raw[4 * j + 3]};
    const int base = ((st * 48 + l * 13) & 8191);
#pragma unroll
    for (int q = 0; q < 12; ++q) raw[q] = img[base + q * 16 + (l & 15)];
    f32x4 fan[2];
    fan[0] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(img) + ((base >> 2) & 2047));
    fan[1] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(img) + (((base >> 2) + 64) & 2047));
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][e], fb[j][e], acc[i][j], 0, 0, 0);
    fa[0] = fan[0] * 1e-30f + fa[0];
    fa[1] = fan[1] * 1e-30f + fa[1];
  }
  __builtin_amdgcn_sched_barrier(0);
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 2; ++i) for (int j = 0; j < 3; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[threadIdx.x] = s;
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
  for (int order = 0; order < 2; ++order) {
    for (int rep = 0; rep < 2; ++rep) {
      if (order == 0) rate6<0><<<1, 256>>>(d, dc); else rate6<1><<<1, 256>>>(d, dc);
    }
    hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
    printf("6-acc wgrad pattern order %s: 1536 MFMAs per wave: %lld ticks (%.2f per MFMA)\n",
           order == 0 ? "(j,e,i)" : "(e,i,j)", hc[0], hc[0] / 1536.0);
  }
  rate6aux<<<1, 256>>>(d, dc);
  rate6aux<<<1, 256>>>(d, dc);
  hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
  printf("6-acc pattern + 14 LDS reads + 12 cvt per step: %lld ticks (%.2f per MFMA)\n", hc[0], hc[0] / 1536.0);
  // the same loop on every CU at once (1024 blocks of 4 waves): clocks under full MFMA load
  float* dbig;
  long long* dcb;
  hipMalloc(&dbig, 1024 * 256 * sizeof(float));
  hipMalloc(&dcb, 1024 * 4 * sizeof(long long));
  for (int rep = 0; rep < 3; ++rep) rate6<0><<<1024, 256>>>(dbig, dcb);
  hipDeviceSynchronize();
  long long hb[4];
  hipMemcpy(hb, dcb, sizeof(hb), hipMemcpyDeviceToHost);
  printf("6-acc pattern, 1024 blocks on all CUs: block 0 %lld ticks (%.2f per MFMA)\n", hb[0], hb[0] / 1536.0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int rep = 0; rep < 20; ++rep) rate6<0><<<1024, 256>>>(dbig, dcb);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  // 1024 blocks x 4 waves x 1536 MFMAs x 2048 FLOP
  printf("  wall: %.3f ms for 20 launches -> %.1f TFLOP/s\n", ms, 20.0 * 1024 * 4 * 1536 * 2048.0 / (ms * 1e-3) / 1e12);
  return 0;
}
