# adam knock-outs (timing only): no kernel-layout shadow re-emission / no moment stores
K = "kernels.h"
SH = "  for (int k = 0; k < n; ++k) write_shadow<T>(a.sp, a.cn, a.sh, i0 + k, p[k]);"
VARIANTS = {
    "adam_base": [],
    "adam_noshadow": [(K, SH, "  for (int k = 0; k < n; ++k) if (p[k] == 12345.f) write_shadow<T>(a.sp, a.cn, a.sh, i0 + k, p[k]);")],
}
