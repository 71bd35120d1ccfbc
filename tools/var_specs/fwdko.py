# conv12_fwd knock-outs (timing only; outputs are wrong): which part sets the per-frame time?
F = "conv1.h"
NO_ACT1_STORE = [(F, "            store4(act1 + ((size_t)f * c1::NPIX + pc) * OC1 + oc, v);\n", "")]
NO_MASK = [(F, "        if (st && lane < 16) mask[(size_t)f * c1::NPIX + pc] = bits;\n        (void)pg;",
            "        if (st && lane < 16 && bits == 0x12345) mask[(size_t)f * c1::NPIX + pc] = bits;\n        (void)pg;")]
NO_PREFETCH = [(F, "    if (f + G < f1) c1_load_frame<T>(x + (size_t)(f + G) * IMG, tid, nv);\n    if (active) {\n      // ---- conv1 -> act1 (HBM + LDS) and its ReLU bit mask ----",
                "    if (active) {\n      // ---- conv1 -> act1 (HBM + LDS) and its ReLU bit mask ----")]
NO_ACT2_STORE = [(F, "          store4(act2 + ((size_t)f * P2 + pc) * OC2 + 16 * wave + 4 * (lane >> 4), v);\n        }\n      }\n    }\n  }\n}",
                  "          if (v[0] == 1234.5f) store4(act2 + ((size_t)f * P2 + pc) * OC2 + 16 * wave + 4 * (lane >> 4), v);\n        }\n      }\n    }\n  }\n}")]
NO_CONV2 = [(F, "        for (int pt = 0; pt < 3; ++pt) acc[pt] = F::mma(a, bq[ks & 1][pt], acc[pt]);",
             "        for (int pt = 0; pt < 3; ++pt) if (ks == 0) acc[pt] = F::mma(a, bq[ks & 1][pt], acc[pt]);")]
VARIANTS = {
    "base": [],
    "ko_act1st": NO_ACT1_STORE,
    "ko_mask": NO_MASK,
    "ko_pref": NO_PREFETCH,
    "ko_act2st": NO_ACT2_STORE,
    "ko_stores": NO_ACT1_STORE + NO_MASK + NO_ACT2_STORE,
    "ko_conv2": NO_CONV2,
}
