# weight prologue issue order rotated per workgroup ((blockIdx >> 3) & 3: differs within an XCD)
# so the CUs of an XCD do not request the same L2 lines in lockstep; same values, same registers
L = "lnc3.h"
C = "conv1.h"
W3_OLD = """  V wa[NT0][NKO];
#pragma unroll
  for (int tt = 0; tt < NT0; ++tt) {
    const int tap = min(NT0 * th + tt, 8);
#pragma unroll
    for (int ko = 0; ko < NKO; ++ko)
      wa[tt][ko] = F::load(w3t + (size_t)(tap * OC2 + 16 * ct + (lane & 15)) * OC3 + ko * KS + kl);
  }
"""
W3_NEW = """  V wa[NT0][NKO];
  auto w3load = [&](auto rc) {
    constexpr int R = decltype(rc)::value;
#pragma unroll
    for (int i = 0; i < NT0 * NKO; ++i) {
      const int jj = (i + R) % (NT0 * NKO), tt = jj / NKO, ko = jj % NKO;
      const int tap = min(NT0 * th + tt, 8);
      wa[tt][ko] = F::load(w3t + (size_t)(tap * OC2 + 16 * ct + (lane & 15)) * OC3 + ko * KS + kl);
    }
  };
  switch ((blockIdx.x >> 3) & 3) {
    case 0: w3load(std::integral_constant<int, 0>{}); break;
    case 1: w3load(std::integral_constant<int, 5>{}); break;
    case 2: w3load(std::integral_constant<int, 10>{}); break;
    default: w3load(std::integral_constant<int, 15>{}); break;
  }
"""
W2_OLD = """#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int kh = py + 2 * (t >> 1), kw = px + 2 * (t & 1);
#pragma unroll
      for (int ks = 0; ks < NKO; ++ks)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
          wb[t][ks][ct] = F::load(w2t + (size_t)((kh * KS2 + kw) * OC1 + 16 * ct + (lane & 15)) * OC2 + ks * KS + kl);
    }
  }"""
W2_NEW = """    auto w2load = [&](auto rc) {
      constexpr int R = decltype(rc)::value;
#pragma unroll
      for (int i = 0; i < 4 * NKO * 2; ++i) {
        const int jj = (i + R) % (4 * NKO * 2), t = jj / (NKO * 2), ks = (jj / 2) % NKO, ct = jj % 2;
        const int kh = py + 2 * (t >> 1), kw = px + 2 * (t & 1);
        wb[t][ks][ct] = F::load(w2t + (size_t)((kh * KS2 + kw) * OC1 + 16 * ct + (lane & 15)) * OC2 + ks * KS + kl);
      }
    };
    switch ((blockIdx.x >> 3) & 3) {
      case 0: w2load(std::integral_constant<int, 0>{}); break;
      case 1: w2load(std::integral_constant<int, 8>{}); break;
      case 2: w2load(std::integral_constant<int, 16>{}); break;
      default: w2load(std::integral_constant<int, 24>{}); break;
    }
  }"""
VARIANTS = {
    "rot_base": [],
    "rot_w3": [(L, W3_OLD, W3_NEW)],
    "rot_both": [(L, W3_OLD, W3_NEW), (C, W2_OLD, W2_NEW)],
}
