# gemm_wg register-ring depth with the row-contiguous Y staging
G = "gemm.h"
PDL = "class Op, int PD = 2>"
VARIANTS = {
    "pd1": [(G, PDL, "class Op, int PD = 1>")],
    "pd2": [],
    "pd3": [(G, PDL, "class Op, int PD = 3>")],
    "pd4": [(G, PDL, "class Op, int PD = 4>")],
}
