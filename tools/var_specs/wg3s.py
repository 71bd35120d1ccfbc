# fp32 merged conv weight gradients at four workgroups per CU: both bodies use 64 x 64 tiles
# (34.8 KB of LDS), so four fit; conv3's split target 256 -> 500 (28 -> 56 splits, 504
# workgroups) fills 1016 of the 1024 slots (conv3's slab 4.1 -> 8.3 MB).
H = "impala.hip"
VARIANTS = {
    "wg3s56": [(H, "  h->sp3 = plan_split((long)N * P3, K3 / 64, 256);",
                "  h->sp3 = plan_split((long)N * P3, K3 / 64, h->bf16 ? 256 : 500);")],
}
