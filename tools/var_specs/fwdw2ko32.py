# timing-only knock-out of the fp32 forward's W2 stream: every k-step reloads k-step 0's
# fragments (L1-resident) instead of streaming 128 KB per frame from L2.  Results are wrong.
C = "conv1.h"
VARIANTS = {
    "fw_base": [],
    "fw_w2same": [(C, "ar[(ks + PD2 - 1) % PD2] = F::load(w2row + (ks + PD2 - 1) * KS);",
                   "ar[(ks + PD2 - 1) % PD2] = F::load(w2row + ((ks + PD2 - 1) & 1) * KS);")],
}
