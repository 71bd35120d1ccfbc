# fp32 FC forward K chunk (gemm_tile<FcFwd>, 32 x 32 tiles): BK 64 (the fp32 cap of BK()) vs
# 128 / 256, i.e. twice / four times the bytes in flight per K chunk, with one or two chunks
# prefetched.  Hypothesis: the kernel is bound by the bytes each CU keeps in flight (a latency-
# bound stream), not by L2 bandwidth (profiles/r05wl: L2-resident operands do not speed up the
# weight-gradient GEMMs).
H = "impala.hip"
L0 = 'gemm_tile<T, 32, 32, BK(256), 2, 2, FcFwd<T>, PF, KA>'
VARIANTS = {
    "fc_bk64": [],
    "fc_bk128_pf2": [(H, L0, 'gemm_tile<T, 32, 32, (sizeof(T) == 4 ? 128 : 256), 2, 2, FcFwd<T>, PF, KA>')],
    "fc_bk128_pf1": [(H, L0, 'gemm_tile<T, 32, 32, (sizeof(T) == 4 ? 128 : 256), 2, 2, FcFwd<T>, 1, KA>')],
    "fc_bk256_pf1": [(H, L0, 'gemm_tile<T, 32, 32, 256, 2, 2, FcFwd<T>, 1, KA>')],
    "fc_bk256_pf2": [(H, L0, 'gemm_tile<T, 32, 32, 256, 2, 2, FcFwd<T>, PF, KA>')],
}
