# knock-outs of reduce_adam_kernel phases (timing only; numerics are wrong except fu_base/unfused)
K = "kernels.h"
SPIN = "    if (__syncthreads_and(ok)) break;"
ST = "      aa.grads[c] = g[j][i];"
SH = "      write_shadow<T>(aa.sp, aa.cn, aa.sh, (size_t)c, p[j][i]);"
VARIANTS = {
    "fu_base": [],
    "fu_nowait": [(K, SPIN, "    if (true) break;")],
    "fu_noshadow": [(K, SH, "")],
    "unfused": [("impala.hip", "  if (const char* e = std::getenv(\"IMPALA_FUSED_UPDATE\")) h->fused_update = e[0] != '0';", "  h->fused_update = false;")],
}
