# Timing-only knock-out for the FC forward (gemm_tile, KACC == 1 loop): every other k-step of
# each chunk skipped (half the MFMAs and half the fragment reads; results garbage).  If fc_fwd
# drops by ~half its MFMA time, the 32 x 32 tiles are bound by their MFMA chains; if not, by the
# chunk loop's staging / barriers / L2 latency.  (Also affects the other KACC == 1 gemm_tile
# users; read fc_fwd only.)
G = "gemm.h"
VARIANTS = {
    "fcf_halfk": [(G, "        for (int kk = 0; kk < BK; kk += F::KSTEP) {\n          V a[TRW], b[TCW];\n          frags(kk, a, b);",
                   "        for (int kk = 0; kk < BK; kk += 2 * F::KSTEP) {\n          V a[TRW], b[TCW];\n          frags(kk, a, b);")],
}
