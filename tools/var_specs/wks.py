# Backward group B (conv1.h C12B32::WKS): conv1 weight gradient split over k-blocks, all taps per
# wave (product) vs one tap per wave over all k-blocks (round 3).
F = "conv1.h"
OLD = "static constexpr bool WKS = true;"
VARIANTS = {"wks_off": [(F, OLD, "static constexpr bool WKS = false;")]}
