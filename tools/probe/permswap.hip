// v_permlane16_swap_b32 / v_permlane32_swap_b32 operand semantics on gfx950, inline asm and
// the clang builtins: a = lane, b = 100 + lane; prints a and b of every 8th lane after a swap.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out, unsigned* in) {
  const unsigned l = in[threadIdx.x];
  unsigned a = l, b = 100 + l;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  out[threadIdx.x] = a;
  out[64 + threadIdx.x] = b;
  unsigned c = l, d = 100 + l;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(c), "+v"(d));
  out[128 + threadIdx.x] = c;
  out[192 + threadIdx.x] = d;
  const auto p = __builtin_amdgcn_permlane16_swap(l, 100 + l, false, false);
  out[256 + threadIdx.x] = p[0];
  out[320 + threadIdx.x] = p[1];
  const auto q = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
  out[384 + threadIdx.x] = q[0];
  out[448 + threadIdx.x] = q[1];
}
int main() {
  unsigned *d, *in;
  (void)hipMalloc(&d, 512 * 4);
  (void)hipMalloc(&in, 64 * 4);
  unsigned h[512];
  for (int i = 0; i < 64; ++i) h[i] = i;
  (void)hipMemcpy(in, h, 64 * 4, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, in);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[8] = {"asm swap16 a", "asm swap16 b", "asm swap32 a", "asm swap32 b",
                       "builtin16 [0]", "builtin16 [1]", "builtin32 [0]", "builtin32 [1]"};
  for (int r = 0; r < 8; ++r) {
    printf("%s:", nm[r]);
    for (int l = 0; l < 64; l += 8) printf(" %u", h[r * 64 + l]);
    printf("\n");
  }
  return 0;
}
