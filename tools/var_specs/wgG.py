H = "impala.hip"
C2 = "    gemm_wg<T, 64, 128, 1, 4, WBM, 2><<<dim3(K2 / 128, 1, h->sp2.S), 512, 0, ss>>>("
C3 = "    gemm_wg<T, 64, 192, 1, 4, WBM, 2><<<dim3(K3 / 192, 1, h->sp3.S), 512, 0, ss>>>("
FC = "    gemm_wg<T, 64, 256, 1, 4, WBM, 1><<<dim3(FLAT / 256, HID / 64, h->spfc.S), 256, 0, ss>>>("
G4 = "(sizeof(T) == 2 ? 4 : 1)"
VARIANTS = {
    "base": [],
    "c2_g4": [(H, C2, f"    gemm_wg<T, 64, 128, 1, 4, 32, {G4}><<<dim3(K2 / 128, 1, h->sp2.S), 256 * {G4}, 0, ss>>>(")],
    "c3_g4": [(H, C3, f"    gemm_wg<T, 64, 192, 1, 4, 32, {G4}><<<dim3(K3 / 192, 1, h->sp3.S), 256 * {G4}, 0, ss>>>(")],
    "fc_g2": [(H, FC, "    gemm_wg<T, 64, 256, 1, 4, 32, (sizeof(T) == 2 ? 2 : 1)><<<dim3(FLAT / 256, HID / 64, h->spfc.S), 256 * (sizeof(T) == 2 ? 2 : 1), 0, ss>>>(")],
}
