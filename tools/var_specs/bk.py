H = "impala.hip"
C3 = "    gemm_tile<T, 64, 64, BK(64), 2, 2><<<persist_grid(h, (long)(cdiv((long)n * P3, 64)) * (1)), 256, 0, st>>>(op, 1);"
D3 = "    gemm_tile<T, 64, 128, BK(64), 1, 4><<<persist_grid(h, (long)(cdiv((long)N * P2, 128)) * (1)), 256, 0, st>>>(op, 1);"
def c3(bk):
    return (H, C3, C3.replace("BK(64)", f"BK({bk})"))
def d3(bk):
    return (H, D3, D3.replace("BK(64)", f"BK({bk})"))
VARIANTS = {"base": [], "c3_96": [c3(96)], "c3_192": [c3(192)], "d3_96": [d3(96)], "d3_192": [d3(192)]}
