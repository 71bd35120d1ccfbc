# Timing-only knock-out for the weight-gradient GEMM body (gemm.h gemm_wg_body): every other
# k-step of each chunk skipped (half the MFMAs and fragment reads; results garbage).  Read
# fc_wgrad_fc_dgrad (the FC weight gradient's 128 long workgroups) and
# conv3_wgrad_conv2_wgrad: how much of each is the MFMA k-loop.
G = "gemm.h"
VARIANTS = {
    "wg_halfk": [(G, "        for (int kk = 0; kk < BM; kk += F::KSTEP) {\n          V a[TRW], b[TCW];",
                  "        for (int kk = 0; kk < BM; kk += 2 * F::KSTEP) {\n          V a[TRW], b[TCW];")],
}
