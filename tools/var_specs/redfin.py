# reduce_grads: the last launch's fin work (loss metrics, step, Adam scalars) knocked out (timing only)
K = "kernels.h"
FIN = "  if (fin && blockIdx.x == 0 && threadIdx.x == 64) {"
SC = "  if (fin && blockIdx.x == 0 && threadIdx.x == 128) {  // step += 1 and its bias corrections"
VARIANTS = {
    "fin_base": [],
    "fin_nometrics": [(K, FIN, "  if (fin && blockIdx.x == 0 && threadIdx.x == 64 && a.B < 0) {")],
    "fin_noscalars": [(K, SC, "  if (fin && blockIdx.x == 0 && threadIdx.x == 128 && a.B < 0) {")],
    "fin_lastblock": [(K, FIN, "  if (fin && blockIdx.x == gridDim.x - 1 && threadIdx.x == 64) {"),
                      (K, SC, "  if (fin && blockIdx.x == gridDim.x - 1 && threadIdx.x == 128) {")],
}
