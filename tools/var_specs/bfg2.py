# bf16 conv weight gradients after the 2-group change: one group (28 KB, more workgroups per CU),
# and 2 groups with more splits (the 508-workgroup split plan was sized for one workgroup per CU)
H = "impala.hip"
L0 = "  constexpr int WG4 = sizeof(T) == 2 ? 2 : 1, WG2 = sizeof(T) == 2 ? 2 : 1;"
C3 = "  h->sp3 = plan_split((long)N * P3, K3 / 64, 256);"
C2 = "  h->sp2 = plan_split((long)N * P2, K2 / 128, 256);"
VARIANTS = {
    "bg2_base": [],
    "bg2_g1": [(H, L0, "  constexpr int WG4 = 1, WG2 = sizeof(T) == 2 ? 2 : 1;")],
    "bg2_s384": [(H, C3, C3.replace("256)", "h->bf16 ? 384 : 256)")), (H, C2, C2.replace("256)", "h->bf16 ? 384 : 256)"))],
    "bg2_s192": [(H, C3, C3.replace("256)", "h->bf16 ? 192 : 256)")), (H, C2, C2.replace("256)", "h->bf16 ? 192 : 256)"))],
}
