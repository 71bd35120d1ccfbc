# launch floor vs grid size: adam with every workgroup returning at entry, 337 vs 64 vs 1 workgroups
K = "kernels.h"
H = "impala.hip"
AD = "__global__ __launch_bounds__(256) void adam_kernel(const AdamArgs a) {"
GR = 'klaunch(h, K_ADAM, "adam", adam_kernel<T>, dim3(cdiv((long)(h->cn.total + 3) / 4, 256))'
VARIANTS = {
    "ae_337": [(K, AD, AD + "\n  if (a.n_part >= 0) return;")],
    "ae_64": [(K, AD, AD + "\n  if (a.n_part >= 0) return;"), (H, GR, 'klaunch(h, K_ADAM, "adam", adam_kernel<T>, dim3(64)')],
    "ae_1": [(K, AD, AD + "\n  if (a.n_part >= 0) return;"), (H, GR, 'klaunch(h, K_ADAM, "adam", adam_kernel<T>, dim3(1)')],
}
