# conv3-tail W3 LDS-DMA prefetch in the last frame iteration, on / off
K = "conv1.h"
VARIANTS = {
    "w3dma_on": [],
    "w3dma_off": [(K, "constexpr bool C3T_W3DMA = true;", "constexpr bool C3T_W3DMA = false;")],
}
