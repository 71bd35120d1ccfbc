H = "impala.hip"
C2 = "    gemm_wg<T, 64, 128, 1, 4, 32, WG4><<<dim3(K2 / 128, 1, h->sp2.S), 256 * WG4, 0, ss>>>("
FC = "    gemm_wg<T, 64, 256, 1, 4, 32, WG2><<<dim3(FLAT / 256, HID / 64, h->spfc.S), 256 * WG2, 0, ss>>>("
VARIANTS = {
    "base": [],
    "c2_16": [(H, C2, C2.replace("32, WG4", "(sizeof(T) == 2 ? 16 : 32), WG4"))],
    "fc_g4_16": [(H, FC, FC.replace("32, WG2><<<", "(sizeof(T) == 2 ? 16 : 32), WG4><<<").replace("256 * WG2", "256 * WG4"))],
}
