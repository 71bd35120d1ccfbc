H = "impala.hip"
FC = "  h->spfc = plan_split(N, (FLAT / 256) * (HID / 64), 96);"
C3 = "  h->sp3 = plan_split((long)N * P3, K3 / 192, 192);"
C2 = "  h->sp2 = plan_split((long)N * P2, K2 / 128, 256);"
VARIANTS = {
    "base": [],
    "fc192": [(H, FC, FC.replace("96)", "192)"))],
    "fc256": [(H, FC, FC.replace("96)", "256)"))],
    "c3_384": [(H, C3, C3.replace("192)", "384)"))],
    "c2_512": [(H, C2, C2.replace("256)", "512)"))],
    "c2_128": [(H, C2, C2.replace("256)", "128)"))],
}
