H = "impala.hip"
C3 = "    gemm_tile<T, 64, 64, BK(96), 2, 2><<<persist_grid(h, (long)(cdiv((long)n * P3, 64)) * (1)), 256, 0, st>>>(op, 1);"
FF = "    gemm_tile<T, 64, 32, BK(256), 2, 2><<<persist_grid(h, (long)cdiv(n, 32) * (HID / 64)), 256, 0, st>>>(op, HID / 64);"
FPT = "    op.frames_per_tile = 64 / P3;"
VARIANTS = {
    "base": [],
    "c3_32": [(H, C3, "    gemm_tile<T, 64, 32, BK(64), 2, 2><<<persist_grid(h, (long)(cdiv((long)n * P3, 32)) * (1)), 256, 0, st>>>(op, 1);"),
              (H, FPT, "    op.frames_per_tile = 32 / P3;")],
    "c3_32_192": [(H, C3, "    gemm_tile<T, 64, 32, BK(192), 2, 2><<<persist_grid(h, (long)(cdiv((long)n * P3, 32)) * (1)), 256, 0, st>>>(op, 1);"),
              (H, FPT, "    op.frames_per_tile = 32 / P3;")],
    "ff_16": [(H, FF, "    gemm_tile<T, 64, 16, (sizeof(T) == 4 ? 64 : 256), 4, 1><<<persist_grid(h, (long)cdiv(n, 16) * (HID / 64)), 256, 0, st>>>(op, HID / 64);")],
}
