# rotated weight staging: each workgroup walks the broadcast weights from a different offset, so
# the CUs of an XCD do not all request the same L2 lines at the same time
F = "conv1.h"
FWD = [
    (F, """#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = (int)threadIdx.x + i * NT;
      if (e < NV1) wv[i] = *reinterpret_cast<const V*>(w1 + (size_t)e * VEC);
      else if (e < NV1 + NV2) wv[i] = *reinterpret_cast<const V*>(w2 + (size_t)(e - NV1) * VEC);
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = (int)threadIdx.x + i * NT;
      if (e < NV1) {""",
     """    constexpr int NVT = NV1 + NV2;
    const int rot = (int)((blockIdx.x * 520u) % NVT);
    auto rix = [&](int i) {
      int r = (int)threadIdx.x + i * NT + rot;
      return r >= NVT ? r - NVT : r;
    };
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      if ((int)threadIdx.x + i * NT < NVT) {
        const int e = rix(i);
        const T* src = e < NV1 ? w1 + (size_t)e * VEC : w2 + (size_t)(e - NV1) * VEC;
        wv[i] = *reinterpret_cast<const V*>(src);
      }
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      if ((int)threadIdx.x + i * NT >= NVT) continue;
      const int e = rix(i);
      if (e < NV1) {"""),
]
BWD = [
    (F, """      const int e = (int)threadIdx.x + i * NT;
      wv[i] = *reinterpret_cast<const V*>(w2 + (size_t)e * VEC);
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = (int)threadIdx.x + i * NT, row = e / (K2 / VEC), c = (e % (K2 / VEC)) * VEC;""",
     """      int e = (int)threadIdx.x + i * NT + (int)((blockIdx.x * 520u) % NWV);
      e = e >= NWV ? e - NWV : e;
      wv[i] = *reinterpret_cast<const V*>(w2 + (size_t)e * VEC);
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      int e = (int)threadIdx.x + i * NT + (int)((blockIdx.x * 520u) % NWV);
      e = e >= NWV ? e - NWV : e;
      const int row = e / (K2 / VEC), c = (e % (K2 / VEC)) * VEC;"""),
]
VARIANTS = {"base": [], "wrot_f": FWD, "wrot_b": BWD, "wrot_fb": FWD + BWD}
