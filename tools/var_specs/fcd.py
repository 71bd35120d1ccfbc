# direct (one-split) FC weight-gradient tile shapes / ring depth
H = "impala.hip"
L = "constexpr int FCD_BR = 32, FCD_BC = 64, FCD_WR = 2, FCD_WC = 2, FCD_G = 4, FCD_PD = 2;"
def V(br, bc, wr, wc, g, pd):
    return [(H, L, f"constexpr int FCD_BR = {br}, FCD_BC = {bc}, FCD_WR = {wr}, FCD_WC = {wc}, FCD_G = {g}, FCD_PD = {pd};")]
VARIANTS = {
    "d32x64": [],
    "d32x64pd3": V(32, 64, 2, 2, 4, 3),
    "d16x64": V(16, 64, 1, 4, 4, 2),
    "d16x64pd3": V(16, 64, 1, 4, 4, 3),
    "d64x64": V(64, 64, 2, 2, 4, 2),
    "d32x128": V(32, 128, 1, 4, 4, 2),
    "slab": [(H, '  h->fc_direct = N <= 8192;', '  h->fc_direct = false;')],
}
