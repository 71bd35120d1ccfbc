# staggered wave groups ("ping-pong"): group 1 runs one barrier phase behind group 0, so the two
# groups' MFMA-heavy and VALU/LDS-heavy phases overlap instead of contending in lock step
F = "conv1.h"
FWD = [
    (F, "  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers of img / a1s are done\n    if (active) c1_stash_frame_rot",
        "  if constexpr (G > 1) if (grp == 1) __builtin_amdgcn_s_barrier();  // stagger\n  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers of img / a1s are done\n    if (active) c1_stash_frame_rot"),
    (F, "          store4(act2 + ((size_t)f * P2 + pc) * OC2 + 16 * wave + 4 * (lane >> 4), v);\n        }\n      }\n    }\n  }\n}",
        "          store4(act2 + ((size_t)f * P2 + pc) * OC2 + 16 * wave + 4 * (lane >> 4), v);\n        }\n      }\n    }\n  }\n  if constexpr (G > 1) if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger\n}"),
]
BWD = [
    (F, "  const int n_it = (f1 - f0 + G - 1) / G;\n  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers are done",
        "  const int n_it = (f1 - f0 + G - 1) / G;\n  if constexpr (G > 1) if (grp == 1) __builtin_amdgcn_s_barrier();  // stagger\n  for (int it = 0; it < n_it; ++it) {\n    const int f = f0 + G * it + grp;\n    const bool active = f < f1;\n    __syncthreads();  // the previous frame's readers are done"),
    (F, "  // conv1 bias: sum each lane's partials over the 16 lanes of its channel group (fixed",
        "  if constexpr (G > 1) if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger\n  // conv1 bias: sum each lane's partials over the 16 lanes of its channel group (fixed"),
]
VARIANTS = {
    "base": [],
    "stag_f": FWD,
    "stag_b": BWD,
    "stag_fb": FWD + BWD,
}
