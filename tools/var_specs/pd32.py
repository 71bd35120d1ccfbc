# fp32 forward weight-stream prefetch depths: conv3 tail W3 ring (PD3) and conv2 W2 ring (PD2)
C = "conv1.h"
P3 = "      constexpr int PD3 = 8;"
P2 = "      constexpr int PD2 = W2REG ? 1 : 4;"
VARIANTS = {
    "base": [],
    "pd3_16": [(C, P3, "      constexpr int PD3 = 16;")],
    "pd3_4": [(C, P3, "      constexpr int PD3 = 4;")],
    "pd2_8": [(C, P2, "      constexpr int PD2 = W2REG ? 1 : 8;")],
    "pd2_2": [(C, P2, "      constexpr int PD2 = W2REG ? 1 : 2;")],
}
