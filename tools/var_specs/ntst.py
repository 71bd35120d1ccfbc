# Non-temporal (streaming, aux = nt) stores for the activations: does the L2 write-back at each
# kernel's end cost the step?  nt_all: store4 (every f32x4 / bf16x4 activation store) and the
# forward's act1 / mask buffer stores; nt_act1: the act1 / mask buffer stores only.
C = "common.h"
S0 = "DEV void store4(float* p, const float v[4]) { *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]}; }"
S1 = "DEV void store4(float* p, const float v[4]) { __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4*>(p)); }"
B0 = "  *reinterpret_cast<bf16x4*>(p) = o;\n}"
B1 = "  __builtin_nontemporal_store(o, reinterpret_cast<bf16x4*>(p));\n}"
A = [("conv1.h", "__builtin_amdgcn_raw_buffer_store_b64(d, rs_act1, gofs + oc * 2, 0, 0);", "__builtin_amdgcn_raw_buffer_store_b64(d, rs_act1, gofs + oc * 2, 0, 2);"),
     ("conv1.h", "__builtin_amdgcn_raw_buffer_store_b128(d, rs_act1, gofs + oc * 4, 0, 0);", "__builtin_amdgcn_raw_buffer_store_b128(d, rs_act1, gofs + oc * 4, 0, 2);")]
VARIANTS = {
    "nt_all": [(C, S0, S1), (C, B0, B1)] + A,
    "nt_act1": A,
}
