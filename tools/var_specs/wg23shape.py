# fp32 weight-gradient tile widths of the merged conv3 + conv2 launch (Wg23Shape<float>):
# conv2 64 x 256 (waves 64 x 64), conv3 64 x 192 (waves 64 x 48), both
O = "ops.h"
BASE = """template <typename T> struct Wg23Shape {
  static constexpr int BC3 = 64, WR3 = 2, WC3 = 2;
  static constexpr int BC2 = 128, WR2 = 1, WC2 = 4;
};"""
def shape(bc3, wr3, wc3, bc2, wr2, wc2):
    return BASE + f"""
template <> struct Wg23Shape<float> {{
  static constexpr int BC3 = {bc3}, WR3 = {wr3}, WC3 = {wc3};
  static constexpr int BC2 = {bc2}, WR2 = {wr2}, WC2 = {wc2};
}};"""
VARIANTS = {
    "ws_base": [],
    "ws_c2w": [(O, BASE, shape(64, 2, 2, 256, 1, 4))],
    "ws_c3w": [(O, BASE, shape(192, 1, 4, 128, 1, 4))],
    "ws_both": [(O, BASE, shape(192, 1, 4, 256, 1, 4))],
}
