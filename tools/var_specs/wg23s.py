# split counts of the merged conv3 + conv2 weight-gradient launch (blocks = 9*S3 + 4*S2)
H = "impala.hip"
C3 = "  h->sp3 = plan_split((long)N * P3, K3 / 64, 256);"
C2 = "  h->sp2 = plan_split((long)N * P2, K2 / 128, 256);"
VARIANTS = {
    "s28_64": [],
    "s14_32": [(H, C3, C3.replace("256)", "128)")), (H, C2, C2.replace("256)", "128)"))],
    "s28_32": [(H, C2, C2.replace("256)", "128)"))],
    "s14_64": [(H, C3, C3.replace("256)", "128)"))],
    "s19_43": [(H, C3, C3.replace("256)", "171)")), (H, C2, C2.replace("256)", "171)"))],
}
