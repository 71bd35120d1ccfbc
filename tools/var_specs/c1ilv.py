# fp32 forward: conv1's second tile pair's MFMAs (72 bf16 passes) interleaved with the first
# pair's epilogue VALU work (sched_group_barrier), instead of the compiler's all-MFMA-first order.
F = "conv1.h"
OLD = "      c1_mma(accA, 0);\n      c1_mma(accB, 2);\n      c1_epi(accA, 0, f);\n      c1_epi(accB, 2, f);\n"


def ilv(m, v, n):
    seq = "".join(f"__builtin_amdgcn_sched_group_barrier(0x008, {m}, 0); __builtin_amdgcn_sched_group_barrier(0x002, {v}, 0); "
                  for _ in range(n))
    return (F, OLD, "      c1_mma(accA, 0);\n      __builtin_amdgcn_sched_barrier(0);\n      c1_mma(accB, 2);\n      c1_epi(accA, 0, f);\n"
            "      if constexpr (sizeof(T) == 4) { " + seq + "}\n      __builtin_amdgcn_sched_barrier(0);\n      c1_epi(accB, 2, f);\n")


VARIANTS = {
    "c1ilv12": [ilv(1, 2, 72)],
    "c1ilv23": [ilv(2, 3, 36)],
}
