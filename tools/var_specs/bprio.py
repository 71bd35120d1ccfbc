# Static wave priority in the fp32 conv12 backward body: group B (waves 4-7, the second-dispatched
# half and the step's bottleneck) at s_setprio 1 before its loop (MI355X_MICROARCH.md, two waves
# per SIMD, item 4); and group A raised instead, for contrast.
C = "conv1.h"
OLD = """    stage(nF > 0 ? f0 : -1, 0, nF > 1 ? f0 + 1 : -1, 1);
    __syncthreads();
    for (int it = 1; it <= nF; ++it) {"""
OLDA = """  if (is_a) {
    // the gather's Z chunk selectors"""
VARIANTS = {
    "bprio1": [(C, OLD, "    __builtin_amdgcn_s_setprio(1);\n" + OLD)],
    "aprio1": [(C, OLDA, "  if (is_a) {\n    __builtin_amdgcn_s_setprio(1);\n    // the gather's Z chunk selectors")],
}
# role 1 (waves 4-7) at priority 1 from the kernel's start: the LayerNorm / conv3-dgrad part too
L = "lnc3.h"
OLDL = """    } else {
      lnc3_body_f32r<1>("""
VARIANTS["r1prio1"] = [(L, OLDL, "    } else {\n      __builtin_amdgcn_s_setprio(1);\n      lnc3_body_f32r<1>(")]
