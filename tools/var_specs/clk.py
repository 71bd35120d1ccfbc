# In-kernel clock of the big fp32 kernels (MI355X_MICROARCH.md 'DVFS give-back' item 6):
# workgroup 0 stamps s_memtime and s_memrealtime (100 MHz) at entry and, after a barrier, at
# exit; the 600th launch of each kernel prints "CLK <id> <shader clocks> <ticks> <GHz>".
# ids: 0 conv12_fwd_s2d, 1 lnc3_conv12_bwd, 2 wgrad23_kernel, 3 head_step (+4: bf16).
C = "common.h"
PROBE = r'''
__device__ int g_clkn[8];
struct ClockProbe {
  int id;
  long long t0, r0;
  __device__ ClockProbe(int i) : id(i) {
    t0 = (long long)__builtin_amdgcn_s_memtime();
    r0 = (long long)__builtin_amdgcn_s_memrealtime();
  }
  __device__ ~ClockProbe() {
    __syncthreads();
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
      const long long t1 = (long long)__builtin_amdgcn_s_memtime(), r1 = (long long)__builtin_amdgcn_s_memrealtime();
      const int n = g_clkn[id];
      if (n == 600) printf("CLK %d %lld %lld %.3f\n", id, t1 - t0, r1 - r0, (double)(t1 - t0) / (double)(r1 - r0) / 10.0);
      g_clkn[id] = n + 1;
    }
  }
};
'''
A = "template <typename T> struct Frag;\n"
VARIANTS = {
    "clk": [
        (C, A, PROBE + A),
        ("conv1.h", "  __shared__ __attribute__((aligned(16))) T smem[C12FLds<T>::ELEMS];\n  conv12_fwd_body<T>(",
         "  ClockProbe cp_(sizeof(T) == 4 ? 0 : 4);\n  __shared__ __attribute__((aligned(16))) T smem[C12FLds<T>::ELEMS];\n  conv12_fwd_body<T>("),
        ("lnc3.h", "  static_assert(lnc3_threads<T>() == 256 * c12_groups<T>(), \"one block shape for both bodies\");\n",
         "  static_assert(lnc3_threads<T>() == 256 * c12_groups<T>(), \"one block shape for both bodies\");\n  ClockProbe cp_(sizeof(T) == 4 ? 1 : 5);\n"),
        ("ops.h", "  __shared__ __attribute__((aligned(16))) T smem[Wg23Cfg<T, G>::SMEM];\n  const int n3",
         "  ClockProbe cp_(sizeof(T) == 4 ? 2 : 6);\n  __shared__ __attribute__((aligned(16))) T smem[Wg23Cfg<T, G>::SMEM];\n  const int n3"),
    ],
}
