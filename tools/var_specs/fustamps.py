# s_memrealtime stamps (10 ns ticks) in reduce_adam_kernel, thread 0 of a few workgroups:
# entry, after the reduction, after publishing, after the sweep, after the Adam stores drained
K = "kernels.h"
COND = "(threadIdx.x == 0 && (blockIdx.x % 50 == 0 || blockIdx.x == gridDim.x - 1))"
def S(i):
    return f"if {COND} st[{i}] = __builtin_amdgcn_s_memrealtime(); "
VARIANTS = {
    "fust": [
        (K, "  // the epoch counter and the step are read first but only waited for after the reduction\n",
            "  long long st[8] = {0}; " + S(0) + "\n"),
        (K, "    for (int i = 0; i < 4; ++i) g[j][i] = acc[i];\n",
            "    for (int i = 0; i < 4; ++i) g[j][i] = acc[i];\n    " + S(1) + "\n"),
        (K, "    __syncthreads();  // part / red are reused by the next unit\n",
            "    __syncthreads();  // part / red are reused by the next unit\n    " + S(2) + "\n"),
        (K, "  float sq = 0.f;\n  if ((int)threadIdx.x < nq) sq += (x[0] + x[1]) + (x[2] + x[3]);",
            "  " + S(3) + "\n  float sq = 0.f;\n  if ((int)threadIdx.x < nq) sq += (x[0] + x[1]) + (x[2] + x[3]);"),
        (K, "      write_shadow<T>(aa.sp, aa.cn, aa.sh, (size_t)c, p[j][i]);\n    }\n}",
            "      write_shadow<T>(aa.sp, aa.cn, aa.sh, (size_t)c, p[j][i]);\n    }\n  __builtin_amdgcn_s_waitcnt(0); " + S(4) + "\n"
            "  if " + COND + ' printf("FUST wg%03d t0 %lld : %lld %lld %lld %lld\\n", (int)blockIdx.x, st[0] % 100000000, st[1]-st[0], st[2]-st[0], st[3]-st[0], st[4]-st[0]);\n}'),
    ],
}
