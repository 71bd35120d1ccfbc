# Timing-only knock-outs of the FC-row adam_kernel (kernels.h, profiles/r05tail): which shadow
# stores are left on its critical path.
#   adam_gen_nosh: the non-FC blocks skip write_shadow (the FC rows still re-emitted via LDS)
#   adam_fc_nosh:  the FC blocks skip their LDS re-emission
K = "kernels.h"
VARIANTS = {
    "adam_gen_nosh": [(K, "    for (int k = 0; k < n; ++k) write_shadow<T>(a.sp, a.cn, a.sh, i0 + k, p[k]);\n  }\n}",
                       "    (void)0;\n  }\n}")],
    "adam_fc_nosh": [(K, "  if (fc) {\n    // canonical j = 4 tid + k", "  if (fc && a.cn.total == 0) {\n    // canonical j = 4 tid + k")],
}
