# ADOPTED in round 4 (conv1.h ar0); kept as the record of the A/B edit.
# fp32 forward: the W2 ring's first three fragments of conv2 loaded at the start of the frame's
# conv1 phase (4.6k clocks earlier) instead of at the top of the conv2 loop, whose first MFMA
# otherwise waits a full L2 round trip every frame.
F = "conv1.h"
VARIANTS = {
    "w2early": [
        (F, "    const bool active = f < f1;\n    if (active) {\n      // ---- conv1",
            "    const bool active = f < f1;\n    V ar0[3];\n    if (active) {\n      // ---- conv1"),
        (F, "      f32x4 accA[2][2], accB[2][2];\n      c1_mma(accA, 0);",
            "      f32x4 accA[2][2], accB[2][2];\n      if constexpr (!W2REG) {\n#pragma unroll\n        for (int d = 0; d < 3; ++d) ar0[d] = F::load(w2row + d * KS);\n      }\n      c1_mma(accA, 0);"),
        (F, "        for (int d = 0; d < PD2 - 1; ++d) ar[d] = F::load(w2row + d * KS);",
            "        for (int d = 0; d < PD2 - 1; ++d) ar[d] = ar0[d];"),
    ],
}
