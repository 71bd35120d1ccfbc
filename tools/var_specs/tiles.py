H = "impala.hip"
C3 = "    gemm_tile<T, 64, 64, BK(96), 2, 2><<<persist_grid(h, (long)(cdiv((long)n * P3, 64)) * (1)), 256, 0, st>>>(op, 1);"
FF = "    gemm_tile<T, 64, 64, BK(256), 2, 2><<<persist_grid(h, (long)cdiv(n, 64) * (HID / 64)), 256, 0, st>>>(op, HID / 64);"
FD = "    gemm_tile<T, 64, 64, BK(128), 2, 2><<<persist_grid(h, (long)(cdiv(N, 64)) * (FLAT / 64)), 256, 0, st>>>(op, FLAT / 64);"
VARIANTS = {
    "base": [],
    "ff_32": [(H, FF, "    gemm_tile<T, 64, 32, BK(256), 2, 2><<<persist_grid(h, (long)cdiv(n, 32) * (HID / 64)), 256, 0, st>>>(op, HID / 64);")],
    "ff_32_128": [(H, FF, "    gemm_tile<T, 64, 32, BK(128), 2, 2><<<persist_grid(h, (long)cdiv(n, 32) * (HID / 64)), 256, 0, st>>>(op, HID / 64);")],
    "fd_32": [(H, FD, "    gemm_tile<T, 64, 32, BK(128), 2, 2><<<persist_grid(h, (long)(cdiv(N, 32)) * (FLAT / 64)), 256, 0, st>>>(op, FLAT / 64);")],
}
