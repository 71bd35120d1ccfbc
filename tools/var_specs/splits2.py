H = "impala.hip"
C3 = "  h->sp3 = plan_split((long)N * P3, K3 / 192, 192);"
C2 = "  h->sp2 = plan_split((long)N * P2, K2 / 128, 256);"
VARIANTS = {
    "base": [],
    "s3_96": [(H, C3, C3.replace("192);", "96);"))],
    "s2_128": [(H, C2, C2.replace("256);", "128);"))],
    "both": [(H, C3, C3.replace("192);", "96);")), (H, C2, C2.replace("256);", "128);"))],
}
