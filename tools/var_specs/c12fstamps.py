# s_memtime stamps in conv12_fwd_s2d<bf16>: workgroup 0, thread 0 of group 0 (fs_g0) or of
# group 1 (fs_g1): entry, weights staged, first frame stashed, then per frame iteration:
# conv1 done / act1 barrier passed / conv2 done / frame barrier passed, end
C = "conv1.h"
def mk(tx):
    COND = f"(sizeof(T) == 2 && blockIdx.x == 0 && threadIdx.x == {tx})"
    def S(i):
        return f"if {COND} st[{i}] = __builtin_amdgcn_s_memtime(); "
    return [
        (C, "  T* img = smem + grp * GSZ;\n  T* a1s = img + IMGSZ;\n",
            "  T* img = smem + grp * GSZ;\n  T* a1s = img + IMGSZ;\n  long long st[24] = {0}; " + S(0) + "\n"),
        (C, "  // consume the bias loads here: waits for them placed inside the loop would",
            "  " + S(1) + "\n  // consume the bias loads here: waits for them placed inside the loop would"),
        (C, "  if (f0 + grp + G < f1) c1_load_frame<T>(x + (size_t)(f0 + grp + G) * IMG, tid, nv);\n  __syncthreads();\n  for (int it = 0; it < n_it; ++it) {",
            "  if (f0 + grp + G < f1) c1_load_frame<T>(x + (size_t)(f0 + grp + G) * IMG, tid, nv);\n  __syncthreads();\n  " + S(2) + "\n  for (int it = 0; it < n_it; ++it) {"),
        (C, "      c1_epi(accB, 2, f);\n    }\n    __syncthreads();  // the act1 tile is complete; the image is free\n",
            "      c1_epi(accB, 2, f);\n    }\n    " + S("3 + 4 * it") + "\n    __syncthreads();  // the act1 tile is complete; the image is free\n    " + S("4 + 4 * it") + "\n"),
        (C, "    __syncthreads();  // the image holds the next frame; the act1 tile is free\n  }\n}",
            "    " + S("5 + 4 * it") + "\n    __syncthreads();  // the image holds the next frame; the act1 tile is free\n    " + S("6 + 4 * it") + "\n  }\n  " + S(20) + "\n  if " + COND + ' { printf("C12F t%d n_it %d :", (int)threadIdx.x, n_it); for (int q = 1; q < 21; ++q) printf(" %lld", st[q] ? st[q] - st[0] : -1); printf("\\n"); }\n}'),
    ]
VARIANTS = {"fs_g0": mk(0), "fs_g1": mk(256)}
