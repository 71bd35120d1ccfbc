C = "conv1.h"
NT_LOAD = (C, "#pragma unroll\n  for (int i = 0; i < 3; ++i) v[i] = reinterpret_cast<const uint4*>(frame)[tid + i * 256];",
              """  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(frame) + tid + i * 256);
    v[i] = uint4{t[0], t[1], t[2], t[3]};
  }""")
VARIANTS = {"base": [], "ntload": [NT_LOAD]}
