# Row stride of the LayerNorm output y (net.h YLD): the FC forward / weight-gradient operand
# rows padded off the 4 KB alignment that puts a 16-row fragment load on one 4 KB stride.
F = "net.h"
OLD = "constexpr int YLD = FLAT;"
VARIANTS = {
    "ypad16": [(F, OLD, "constexpr int YLD = FLAT + 16;")],
    "ypad64": [(F, OLD, "constexpr int YLD = FLAT + 64;")],
}
