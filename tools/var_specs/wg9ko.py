# Timing-only bound for an exact bf16x9 fp32 weight gradient (gemm.h gemm_wg_body, fp32): the
# k-loop's 4 v_mfma_f32_16x16x4_f32 per 16-deep k-step (128 cycles) replaced by 4 or 5
# v_mfma_f32_16x16x32_bf16 on the same fragment registers bit-cast (9 per 32-deep k-step, 144
# cycles against 256), LDS layout and loads unchanged (plus 4 v_and per fragment to keep the
# bit-cast values finite).  Results garbage: the time the conv
# weight gradients would take if their MFMAs ran at the bf16x9 rate with no extra bytes.
G = "gemm.h"
OLD = """            b[j] = lds_frag_k_sw(Ys + kk * LDY + (wc * TCW + j) * 16, LDY, lane);
#pragma unroll
          for (int i = 0; i < TRW; ++i)
#pragma unroll
            for (int j = 0; j < TCW; ++j) acc[i][j] = F::mma(a[i], b[j], acc[i][j]);"""
NEW = """            b[j] = lds_frag_k_sw(Ys + kk * LDY + (wc * TCW + j) * 16, LDY, lane);
          if constexpr (sizeof(T) == 4) {
            const int nb = (kk / F::KSTEP) % 2 == 0 ? 5 : 4;
            // keep the bit-cast bf16 values finite (exponent <= 126): 4 v_and per fragment
            bf16x8 ab[TRW], bb[TCW];
#pragma unroll
            for (int i = 0; i < TRW; ++i) {
              uint4 x = __builtin_bit_cast(uint4, a[i]);
              x.x &= 0x3F7F3F7Fu; x.y &= 0x3F7F3F7Fu; x.z &= 0x3F7F3F7Fu; x.w &= 0x3F7F3F7Fu;
              ab[i] = __builtin_bit_cast(bf16x8, x);
            }
#pragma unroll
            for (int j = 0; j < TCW; ++j) {
              uint4 x = __builtin_bit_cast(uint4, b[j]);
              x.x &= 0x3F7F3F7Fu; x.y &= 0x3F7F3F7Fu; x.z &= 0x3F7F3F7Fu; x.w &= 0x3F7F3F7Fu;
              bb[j] = __builtin_bit_cast(bf16x8, x);
            }
#pragma unroll
            for (int u = 0; u < 5; ++u)
              if (u < nb)
#pragma unroll
                for (int i = 0; i < TRW; ++i)
#pragma unroll
                  for (int j = 0; j < TCW; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab[i], bb[j], acc[i][j], 0, 0, 0);
          } else {
#pragma unroll
          for (int i = 0; i < TRW; ++i)
#pragma unroll
            for (int j = 0; j < TCW; ++j) acc[i][j] = F::mma(a[i], b[j], acc[i][j]);
          }"""
VARIANTS = {"wg_bf9": [(G, OLD, NEW)]}
