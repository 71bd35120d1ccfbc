# weight-gradient tile / split variants: fewer fp32 partial slabs (smaller tiles, fewer splits)
F = "impala.hip"
FC_OLD = ("gemm_wg<T, 64, 256, 1, 4, 32, WG2, FcWgrad<T>>,\n                        dim3(FLAT / 256, HID / 64, h->spfc.S)",
          "  h->spfc = plan_split(N, (FLAT / 256) * (HID / 64), 96);")
FC32 = [(F, FC_OLD[0], "gemm_wg<T, 32, 32, 2, 2, 32, WG2, FcWgrad<T>>,\n                        dim3(FLAT / 32, HID / 32, h->spfc.S)"),
        (F, FC_OLD[1], "  h->spfc = plan_split(N, (FLAT / 32) * (HID / 32), 256);")]
C3_64 = [(F, "gemm_wg<T, 64, 192, 1, 4, 32, WG4, Conv3Wgrad<T>>,\n                        dim3(K3 / 192, 1, h->sp3.S)",
          "gemm_wg<T, 64, 64, 2, 2, 32, WG4, Conv3Wgrad<T>>,\n                        dim3(K3 / 64, 1, h->sp3.S)"),
         (F, "  h->sp3 = plan_split((long)N * P3, K3 / 192, 192);", "  h->sp3 = plan_split((long)N * P3, K3 / 64, 256);")]
C2_64 = [(F, "gemm_wg<T, 64, 128, 1, 4, 32, WG4, Conv2Wgrad<T>>,\n                        dim3(K2 / 128, 1, h->sp2.S)",
          "gemm_wg<T, 64, 64, 2, 2, 32, WG4, Conv2Wgrad<T>>,\n                        dim3(K2 / 64, 1, h->sp2.S)"),
         (F, "  h->sp2 = plan_split((long)N * P2, K2 / 128, 256);", "  h->sp2 = plan_split((long)N * P2, K2 / 64, 256);")]
VARIANTS = {
    "base": [],
    "fc32": FC32,
    "c3_64": C3_64,
    "c2_64": C2_64,
    "all3": FC32 + C3_64 + C2_64,
}
