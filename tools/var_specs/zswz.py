# Backward Z tile (conv1.h C12B32): XOR-swizzled 64-float rows (product) vs the round-3 68-float pitch.
F = "conv1.h"
OLD = "static constexpr bool ZSWZ = true;"
VARIANTS = {"zpitch68": [(F, OLD, "static constexpr bool ZSWZ = false;")]}
