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
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

#define WAVE 64
// IMPALA_AB=1 (python -m impala_amd.build --ab) also compiles the measured-slower alternative
// kernels kept for A/B runs (fc_fwd_splitk_f32 / fc_fwd_wsplit_f32, fwd_chain_kernel,
// reduce_adam_kernel, wgrad23r_kernel); the product library is built without them, and asking
// a non-A/B library for one (IMPALA_FC_SPLITK, IMPALA_FWD_CHAIN, IMPALA_FUSED_UPDATE,
// IMPALA_EARLY_RED) fails impala_create with IMPALA_E_UNSUPPORTED.
#ifndef IMPALA_AB
#define IMPALA_AB 0
#endif
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
  // MFMA e (0..NE-1) of a k-step alone.  Loops that update several independent accumulators
  // issue element e of every accumulator before element e + 1 of any: a 16x16x4 f32 MFMA issues
  // every 32 cycles but one that reads the previous one's result waits 40, so mma()'s chain of
  // four on one accumulator stalls 3 x 8 cycles per k-step (r03 stamps: conv phases at 82 % of
  // the MFMA issue rate).  Every accumulator still sees the same MFMAs in the same order, so the
  // results are bit-identical to mma().
  static constexpr int NE = 4;
  static DEV f32x4 mma_e(int e, const vec& a, const vec& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], b[e], c, 0, 0, 0);
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
  static constexpr int NE = 1;  // one MFMA per k-step (see Frag<float>::mma_e)
  static DEV f32x4 mma_e(int, const vec& a, const vec& b, f32x4 c) { return mma(a, b, c); }
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

// An fp32 value split exactly into three bf16 terms x = hi + mid + lo (round-to-nearest 8-bit
// pieces of its 24-bit significand: the residual after hi has <= 16 significant bits, after
// mid <= 8); a product of a term with a bf16-exact value (conv1's image bytes) is exact in fp32.
DEV void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

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
// two floats -> two bf16 (round to nearest even, as a (__bf16) cast) packed in one dword
DEV int pack_bf16x2(float a, float b) {
  bf16x2 v;
  v[0] = (__bf16)a;
  v[1] = (__bf16)b;
  return __builtin_bit_cast(int, v);
}
DEV void load4(const float* p, float v[4]) {
  f32x4 x = *reinterpret_cast<const f32x4*>(p);
  v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
}
DEV void load4(const __bf16* p, float v[4]) {
  bf16x4 x = *reinterpret_cast<const bf16x4*>(p);
  v[0] = (float)x[0]; v[1] = (float)x[1]; v[2] = (float)x[2]; v[3] = (float)x[3];
}

// ---- cross-lane moves without the LDS crossbar: DPP within rows of 16 lanes, the gfx950
// permlane swaps across rows.  Every reduction below combines symmetric pairs only, so all
// lanes end with the bit-identical result (and runs are deterministic). ----
template <int CTRL> DEV float dppf(float v) {  // lanes without a source read 0
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL> DEV uint32_t dppu(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
enum : int { DPP_QP_1032 = 0xB1, DPP_QP_2301 = 0x4E, DPP_ROW_MIRROR = 0x140,
             DPP_ROW_HALF_MIRROR = 0x141, DPP_WAVE_SHL1 = 0x130, DPP_WAVE_SHR1 = 0x138 };
// x[lane ^ 16] (resp. ^ 32) exchanges across rows with v_permlane16/32_swap_b32.  Inline asm
// with two read-write operands keeps the two copies in distinct registers: the builtin lets the
// compiler tie both operands to one register, which swaps a register with itself.  The s_nop
// covers the VALU-write -> permlane-read hazard the compiler cannot see through inline asm.
// (Operand semantics checked on gfx950 by tools/probe/permswap.hip.)
DEV void swap16(uint32_t& a, uint32_t& b) { asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b)); }
DEV void swap32(uint32_t& a, uint32_t& b) { asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b)); }
DEV float xor16_sum(float v) {  // v[lane & ~16] + v[lane | 16] on every lane
  uint32_t a = __builtin_bit_cast(uint32_t, v), b = a;
  swap16(a, b);
  return __builtin_bit_cast(float, a) + __builtin_bit_cast(float, b);
}
DEV float xor32_sum(float v) {
  uint32_t a = __builtin_bit_cast(uint32_t, v), b = a;
  swap32(a, b);
  return __builtin_bit_cast(float, a) + __builtin_bit_cast(float, b);
}
// Four values reduced over the four rows at once (3 swaps, 3 adds, instead of 4 x 2 of each):
// row r of the result holds ((x[row 0] + x[row 1]) + (x[row 2] + x[row 3])) of x = a, b, c, d for
// r = 0, 1, 2, 3 -- the value and the order of xor32_sum(xor16_sum(x)).
DEV float rows_sum4(float a, float b, float c, float d) {
  // one asm block: its inputs come straight from MFMAs, whose results a following VALU /
  // permlane may only read after the XDL write latency (the leading 20 wait states; the
  // compiler does not insert them for inline asm), and the adds -> permlane32 read hazard
  // (s_nop 1).  Rows after the swaps: a = [a0 b0 a2 b2], b = [a1 b1 a3 b3]; after the adds and
  // the xor-32 swap, a = [a01 b01 c01 d01], c = [a23 b23 c23 d23].
  asm volatile(
      "s_nop 7\n\ts_nop 7\n\ts_nop 3\n\t"
      "v_permlane16_swap_b32 %0, %1\n\t"
      "v_permlane16_swap_b32 %2, %3\n\t"
      "s_nop 1\n\t"
      "v_add_f32 %0, %0, %1\n\t"
      "v_add_f32 %2, %2, %3\n\t"
      "s_nop 1\n\t"
      "v_permlane32_swap_b32 %0, %2\n\t"
      "s_nop 1\n\t"
      "v_add_f32 %0, %0, %2\n\t"
      "s_nop 1"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  return a;
}
DEV uint32_t xor16_or(uint32_t v) {
  uint32_t a = v, b = v;
  swap16(a, b);
  return a | b;
}
DEV uint32_t xor32_or(uint32_t v) {
  uint32_t a = v, b = v;
  swap32(a, b);
  return a | b;
}
// sum over the 16 lanes of each row (all 16 lanes get the row sum)
DEV float row16_sum(float v) {
  v += dppf<DPP_QP_1032>(v);
  v += dppf<DPP_QP_2301>(v);
  v += dppf<DPP_ROW_HALF_MIRROR>(v);
  v += dppf<DPP_ROW_MIRROR>(v);
  return v;
}
DEV float row16_max(float v) {
  v = fmaxf(v, dppf<DPP_QP_1032>(v));
  v = fmaxf(v, dppf<DPP_QP_2301>(v));
  v = fmaxf(v, dppf<DPP_ROW_HALF_MIRROR>(v));
  return fmaxf(v, dppf<DPP_ROW_MIRROR>(v));
}
// over the 4 lanes of each quad (all four get the bit-identical result)
DEV float quad_sum(float v) {
  v += dppf<DPP_QP_1032>(v);
  return v + dppf<DPP_QP_2301>(v);
}
DEV float quad_max(float v) {
  v = fmaxf(v, dppf<DPP_QP_1032>(v));
  return fmaxf(v, dppf<DPP_QP_2301>(v));
}
DEV float wave_sum(float v) { return xor32_sum(xor16_sum(row16_sum(v))); }
DEV float wave_max(float v) {
  v = fmaxf(v, dppf<DPP_QP_1032>(v));
  v = fmaxf(v, dppf<DPP_QP_2301>(v));
  v = fmaxf(v, dppf<DPP_ROW_HALF_MIRROR>(v));
  v = fmaxf(v, dppf<DPP_ROW_MIRROR>(v));
  uint32_t a = __builtin_bit_cast(uint32_t, v), b = a;
  swap16(a, b);
  v = fmaxf(__builtin_bit_cast(float, a), __builtin_bit_cast(float, b));
  a = __builtin_bit_cast(uint32_t, v);
  b = a;
  swap32(a, b);
  return fmaxf(__builtin_bit_cast(float, a), __builtin_bit_cast(float, b));
}
// lane i reads lane i + 1 (lane 63 reads 0): __shfl_down(v, 1) without the LDS crossbar
DEV float shift_down1(float v) { return dppf<DPP_WAVE_SHL1>(v); }
// lane i reads lane i - 1 (lane 0 reads 0): __shfl_up(v, 1)
DEV float shift_up1(float v) { return dppf<DPP_WAVE_SHR1>(v); }

// exact (erf) GELU, models/models.py:68 nn.GELU() default approximate='none'
DEV float gelu_f(float z) { return 0.5f * z * (1.f + erff(z * 0.70710678118654752440f)); }
DEV float gelu_grad(float z) {
  const float cdf = 0.5f * (1.f + erff(z * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * expf(-0.5f * z * z);
  return cdf + z * pdf;
}
// GELU and its derivative from one erf (the FC forward epilogue keeps gelu'(z) for the backward)
DEV void gelu_fwd_grad(float z, float& h, float& g) {
  const float e = erff(z * 0.70710678118654752440f);
  h = 0.5f * z * (1.f + e);
  g = 0.5f * (1.f + e) + z * (0.39894228040143267794f * expf(-0.5f * z * z));
}
