# after the wave-parallel metrics: is the step / Adam-scalar lane (double pow) the reduce tail?
K = "kernels.h"
SC = "  if (fin && blockIdx.x == 0 && threadIdx.x == 128) {  // step += 1 and its bias corrections"
VARIANTS = {
    "fin2_base": [],
    "fin2_noscalars": [(K, SC, "  if (fin && blockIdx.x == 0 && threadIdx.x == 128 && a.B < 0) {")],
}
