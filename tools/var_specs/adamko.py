# Timing-only knock-outs of adam_kernel (kernels.h): what its 6.5-7 us go to.
#   adam_nosh:  no kernel-layout (shadow) weight stores
#   adam_nonorm: no norm-partial loads / sum (coef = 1)
#   adam_both:  neither
K = "kernels.h"
SH = ("  for (int k = 0; k < n; ++k) write_shadow<T>(a.sp, a.cn, a.sh, i0 + k, p[k]);\n}",
      "  (void)0;\n}")
NO = ("  for (int q0 = threadIdx.x; q0 < nq; q0 += 256 * 4) {\n    f32x4 x[4];",
      "  for (int q0 = threadIdx.x; q0 < nq * 0; q0 += 256 * 4) {\n    f32x4 x[4];")
VARIANTS = {
    "adam_nosh": [(K,) + SH],
    "adam_nonorm": [(K,) + NO],
    "adam_both": [(K,) + SH, (K,) + NO],
}
