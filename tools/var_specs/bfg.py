# bf16 weight-gradient group counts: wgrad23_kernel<bf16, 4> declares 112 KB of LDS (4 groups
# of 64 x 128 tiles, 32-row double-buffered chunks), so its 508 workgroups run one per CU in
# about two rounds; fc_bwd_kernel<bf16, 2> 108 KB likewise.  G = 2 / 1 halves them (two
# workgroups per CU).
H = "impala.hip"
L0 = "  constexpr int WG4 = sizeof(T) == 2 ? 4 : 1, WG2 = sizeof(T) == 2 ? 2 : 1;"
VARIANTS = {
    "bg_base": [],
    "bg_wg2": [(H, L0, "  constexpr int WG4 = sizeof(T) == 2 ? 2 : 1, WG2 = sizeof(T) == 2 ? 2 : 1;")],
    "bg_fc1": [(H, L0, "  constexpr int WG4 = sizeof(T) == 2 ? 4 : 1, WG2 = 1;")],
    "bg_both": [(H, L0, "  constexpr int WG4 = sizeof(T) == 2 ? 2 : 1, WG2 = 1;")],
}
