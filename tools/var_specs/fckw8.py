# fp32 FC forward KW tile shapes on 8 waves (impala.hip FCF_BR x FCF_BC, FCF_NW = 8):
# the product 32 x 48 (216 tiles) against 16 x 80 (256 tiles, all CUs) and 16 x 96 (224).
H = "impala.hip"
OLD = "constexpr int FCF_BR = 16, FCF_BC = 80;"
VARIANTS = {
    "fckw8_16x80": [(H, OLD, "constexpr int FCF_BR = 16, FCF_BC = 80;")],
    "fckw8_32x32": [(H, OLD, "constexpr int FCF_BR = 32, FCF_BC = 32;")],
}
