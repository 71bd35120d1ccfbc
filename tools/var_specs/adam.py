K = "kernels.h"
VARIANTS = {
    "base": [],
    "powf": [(K, "    const double bc1 = 1.0 - pow(a.b1, stepd), bc2 = 1.0 - pow(a.b2, stepd);",
                 "    const double bc1 = 1.0 - (double)powf((float)a.b1, (float)stepd), bc2 = 1.0 - (double)powf((float)a.b2, (float)stepd);")],
    "noshadow": [(K, "  for (int k = 0; k < n; ++k) write_shadow<T>(a.sp, a.cn, a.sh, i0 + k, p[k]);\n}\n", "}\n")],
    "nonorm": [(K, "  for (int q = threadIdx.x; q < a.n_part; q += 256) s += a.sumsq_part[q];", "")],
}
