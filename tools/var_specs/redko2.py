# reduce_grads / adam floor: empty kernels (timing only)
K = "kernels.h"
RG = "__global__ __launch_bounds__(256) void reduce_grads_kernel(const RedArgs a, int s_lo, int fin) {"
AD = "__global__ __launch_bounds__(256) void adam_kernel(const AdamArgs a) {"
VARIANTS = {
    "red_base": [],
    "red_empty": [(K, RG, RG + "\n  if (s_lo >= 0) return;")],
    "adam_empty": [(K, AD, AD + "\n  if (a.n_part >= 0) return;")],
    "red_1wg": [(K, RG, RG + "\n  if (blockIdx.x > 0) return;")],
}
