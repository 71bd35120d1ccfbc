# fp32 FC weight-gradient split count (the slab the reduction reads: 1 MB per split):
# 256 workgroups (16 splits, default) against 128 / 64
H = "impala.hip"
A = "h->spfc = plan_split(N, (FLAT / 256) * (HID / 64), h->bf16 ? 96 : 256);"
VARIANTS = {
    "sf_256": [],
    "sf_128": [(H, A, A.replace("h->bf16 ? 96 : 256", "h->bf16 ? 96 : 128"))],
    "sf_64": [(H, A, A.replace("h->bf16 ? 96 : 256", "h->bf16 ? 96 : 64"))],
}
