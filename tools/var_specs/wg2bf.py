# bf16 conv2 weight-gradient tile in the merged launch (ops.h Wg2Tile): 64 x 64 on 2 x 2 waves
# like fp32 (512 workgroups of conv3's size) instead of 64 x 128 on 1 x 4.
O = "  static constexpr int BC = sizeof(T) == 4 ? 64 : 128, WR = sizeof(T) == 4 ? 2 : 1, WC = 4 / WR;"
VARIANTS = {"wg2bf_64": [("ops.h", O, "  static constexpr int BC = 64, WR = 2, WC = 4 / WR;")]}
