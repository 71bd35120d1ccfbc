// Shared device helpers for the IMPALA learner kernels (gfx950 / CDNA4 only).
//
// Precision model: conv / linear operands are stored in the compute type T (float for the
// fp32 parity mode, __bf16 for the perf mode); every MFMA accumulates in fp32; LayerNorm
// statistics, GELU pre-activations, the loss head, gradients and Adam state are fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

#define WAVE 64
#define DEV __device__ __forceinline__

// ---------------------------------------------------------------------------------------
// Fragment traits.  For a 16x16 output tile every lane owns KPL contiguous k-elements of its
// A row (row = lane & 15) and of its B column (col = lane & 15), starting at
// k0 = KPL * (lane >> 4) inside a K-step of KSTEP = 4 * KPL.
//   bf16: KPL = 8  -> one v_mfma_f32_16x16x32_bf16 per K-step.
//   f32 : KPL = 4  -> four v_mfma_f32_16x16x4_f32, MFMA i consumes element i of every lane's
//         float4, i.e. k-set {i, 4+i, 8+i, 12+i}; A and B use the same permutation so the
//         product is the full K-step sum (exact f32 fma chain per MFMA).
// C/D map (both): col = lane & 15, row = 4 * (lane >> 4) + reg.
// ---------------------------------------------------------------------------------------
template <typename T> struct Frag;

template <> struct Frag<float> {
  static constexpr int KPL = 4;
  static constexpr int KSTEP = 16;
  typedef f32x4 vec;
  static DEV vec zero() { return vec{0.f, 0.f, 0.f, 0.f}; }
  static DEV f32x4 mma(const vec& a, const vec& b, f32x4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
    return c;
  }
  static DEV vec load(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
  static DEV vec from_u8(uint32_t w) {  // 4 bytes -> 4 floats (raw 0..255)
    return vec{(float)(w & 255u), (float)((w >> 8) & 255u), (float)((w >> 16) & 255u),
               (float)(w >> 24)};
  }
};

template <> struct Frag<__bf16> {
  static constexpr int KPL = 8;
  static constexpr int KSTEP = 32;
  typedef bf16x8 vec;
  static DEV vec zero() {
    vec v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (__bf16)0.f;
    return v;
  }
  static DEV f32x4 mma(const vec& a, const vec& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static DEV vec load(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
  static DEV vec from_u8_2(uint32_t lo, uint32_t hi) {  // 8 bytes -> 8 bf16 (exact: <= 255)
    vec v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (__bf16)(float)((lo >> (8 * i)) & 255u);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[4 + i] = (__bf16)(float)((hi >> (8 * i)) & 255u);
    return v;
  }
};

// Workgroups are dispatched round-robin over the 8 XCDs, each with its own L2.  Remap a linear
// dispatch id so that consecutive work items (which share an operand: the row tiles of one
// column tile, the column tiles of one split) run on the same XCD and share its L2.
DEV int xcd_swizzle(int bid, int nb) {
  constexpr int NXCD = 8;
  const int x = bid % NXCD, q = nb / NXCD, r = nb % NXCD;
  return x * q + min(x, r) + bid / NXCD;
}

template <typename T> DEV T to_t(float x) { return (T)x; }
template <typename T> DEV float to_f(T x) { return (float)x; }

// store 4 consecutive values (rows r..r+3 of one output column) to a channels-last row
DEV void store4(float* p, const float v[4]) { *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]}; }
DEV void store4(__bf16* p, const float v[4]) {
  bf16x4 o;
  o[0] = (__bf16)v[0]; o[1] = (__bf16)v[1]; o[2] = (__bf16)v[2]; o[3] = (__bf16)v[3];
  *reinterpret_cast<bf16x4*>(p) = o;
}
DEV void load4(const float* p, float v[4]) {
  f32x4 x = *reinterpret_cast<const f32x4*>(p);
  v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
}
DEV void load4(const __bf16* p, float v[4]) {
  bf16x4 x = *reinterpret_cast<const bf16x4*>(p);
  v[0] = (float)x[0]; v[1] = (float)x[1]; v[2] = (float)x[2]; v[3] = (float)x[3];
}

DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// exact (erf) GELU, models/models.py:68 nn.GELU() default approximate='none'
DEV float gelu_f(float z) { return 0.5f * z * (1.f + erff(z * 0.70710678118654752440f)); }
DEV float gelu_grad(float z) {
  const float cdf = 0.5f * (1.f + erff(z * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * expf(-0.5f * z * z);
  return cdf + z * pdf;
}
