F = "conv1.h"
VARIANTS = {
    "base": [],
    "no_dgrad": [(F, "for (int nt = 0; nt < 4 && active; ++nt) {", "for (int nt = 0; nt < 0 && active; ++nt) {")],
    "no_wgrad": [(F, "    for (int kk = 0; kk < c1::NPAD; kk += KS) {\n      V a[2], b[3];\n#pragma unroll\n      for (int i = 0; i < 2; ++i) a[i] = lds_frag_k(dyt + kk",
                  "    for (int kk = 0; kk < 0; kk += KS) {\n      V a[2], b[3];\n#pragma unroll\n      for (int i = 0; i < 2; ++i) a[i] = lds_frag_k(dyt + kk")],
    "no_w2load": [(F, "        for (int j = 0; j < KPL; ++j) v[j] = src[(size_t)j * K2];", "        for (int j = 0; j < KPL; ++j) v[j] = (T)(float)(lane + j);")],
    "no_stash": [(F, "    if (active) {\n    c1_stash_frame<T>(img, tid, nv);", "    if (active) {\n    if (N < 0) c1_stash_frame<T>(img, tid, nv);")],
}
