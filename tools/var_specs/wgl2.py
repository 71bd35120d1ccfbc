# Timing-only knock-outs of the weight-gradient GEMMs' operand traffic (gemm_wg_body, shared by
# wgrad23 and the FC weight gradient): every chunk load of X and/or Y re-reads the split's first
# 64 rows (L2-resident) instead of streaming the split's rows.  Results are garbage; the
# question is how much of wgrad23's 51 us is the L2 / MALL -> CU stream.
G = "gemm.h"
X0 = "const uint32_t off = (uint32_t)(min(m, m_end - 1) * op.x_ld * (int)sizeof(T) + xcol[i]);"
X1 = "const uint32_t off = (uint32_t)((m_beg + (min(m, m_end - 1) & 63)) * op.x_ld * (int)sizeof(T) + xcol[i]);"
Y0 = "const uint32_t yr = m < m_end ? (uint32_t)(op.y_roff(min(m, m_end - 1)) * (int)sizeof(T)) : (uint32_t)OOB;"
Y1 = "const uint32_t yr = m < m_end ? (uint32_t)(op.y_roff(m_beg + (min(m, m_end - 1) & 63)) * (int)sizeof(T)) : (uint32_t)OOB;"
VARIANTS = {
    "wl_base": [],
    "wl_x": [(G, X0, X1)],
    "wl_y": [(G, Y0, Y1)],
    "wl_xy": [(G, X0, X1), (G, Y0, Y1)],
}
