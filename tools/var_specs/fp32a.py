# fp32 quick wins: gemm_tile K chunk, FC dgrad chunk, weight-gradient groups
H = "impala.hip"
O = "ops.h"
BKL = "#define BK(kb) (sizeof(T) == 4 ? 32 : (kb))"
WGL = "  constexpr int WG4 = sizeof(T) == 2 ? 4 : 1, WG2 = sizeof(T) == 2 ? 2 : 1;"
DBL = "DBK = sizeof(T) == 2 ? 128 : 32;"
VARIANTS = {
    "base": [],
    "bk_same": [(H, BKL, "#define BK(kb) (kb)")],
    "bk_same_d128": [(H, BKL, "#define BK(kb) (kb)"), (O, DBL, "DBK = 128;")],
    "bk64_d64": [(H, BKL, "#define BK(kb) (sizeof(T) == 4 ? ((kb) < 64 ? (kb) : 64) : (kb))"), (O, DBL, "DBK = sizeof(T) == 2 ? 128 : 64;")],
    "bk128_d128": [(H, BKL, "#define BK(kb) (sizeof(T) == 4 ? ((kb) < 128 ? (kb) : 128) : (kb))"), (O, DBL, "DBK = 128;")],
    "wg2": [(H, WGL, "  constexpr int WG4 = sizeof(T) == 2 ? 4 : 2, WG2 = sizeof(T) == 2 ? 2 : 1;")],
    "wg3": [(H, WGL, "  constexpr int WG4 = sizeof(T) == 2 ? 4 : 3, WG2 = sizeof(T) == 2 ? 2 : 1;")],
}
