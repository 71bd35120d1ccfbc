# Timing-only knock-out of the fp32 forward's W2 stream (conv1.h conv12_fwd_body, !W2REG): each
# wave re-reads the first 8 k-steps of its W2 rows (8 KB per wave, L1-resident) instead of all
# 32 (32 KB per wave per frame from L2; 128 KB per CU per frame, 640 KB per CU per step).  The
# results are garbage.  Is the per-CU load path (~11-15 B/clk) the conv2 phase's bound?
C = "conv1.h"
VARIANTS = {
    "w2_base": [],
    "w2_l1": [(C, "          if (ks + PD2 - 1 < NKS2) ar[(ks + PD2 - 1) % PD2] = F::load(w2row + (ks + PD2 - 1) * KS);",
                  "          if (ks + PD2 - 1 < NKS2) ar[(ks + PD2 - 1) % PD2] = F::load(w2row + ((ks + PD2 - 1) & 7) * KS);")],
}
