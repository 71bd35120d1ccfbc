# Entry time (s_memrealtime, 100 MHz, device-global) of wave 0 and wave 4 (group 1) of a few
# conv12_fwd workgroups, and s_memtime stamps of the head_step phases (wg 0/0, thread 0)
C = "conv1.h"
H = "head.h"
CF = "(sizeof(T) == 2 && (blockIdx.x == 0 || blockIdx.x == 100 || blockIdx.x == 255) && (threadIdx.x == 0 || threadIdx.x == 256))"
CH = "(sizeof(T) == 2 && !PPO && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)"
def SH(i):
    return f"if {CH} st[{i}] = __builtin_amdgcn_s_memtime(); "
VARIANTS = {
    "entry": [
        (C, "  T* img = smem + grp * GSZ;\n  T* a1s = img + IMGSZ;\n",
            "  T* img = smem + grp * GSZ;\n  T* a1s = img + IMGSZ;\n  const long long rt0 = __builtin_amdgcn_s_memrealtime(); const long long mt0 = __builtin_amdgcn_s_memtime();\n"),
        (C, "  // consume the bias loads here: waits for them placed inside the loop would",
            "  if " + CF + ' { const long long rt1 = __builtin_amdgcn_s_memrealtime(); printf("C12FE wg%d t%d rt0 %lld rt1 %lld mt %lld\\n", (int)blockIdx.x, (int)threadIdx.x, rt0 % 1000000, rt1 % 1000000, __builtin_amdgcn_s_memtime() - mt0); }\n  // consume the bias loads here: waits for them placed inside the loop would'),
        (H, "  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n  const int T_ = a.T, S = a.S;",
            "  long long st[8] = {0}; " + SH(0) + "\n  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n  const int T_ = a.T, S = a.S;"),
        (H, "  for (int e = tid; e < 64 * LDD / VEC; e += 256) *reinterpret_cast<V*>(dHs + e * VEC) = F::zero();\n  __syncthreads();\n",
            "  for (int e = tid; e < 64 * LDD / VEC; e += 256) *reinterpret_cast<V*>(dHs + e * VEC) = F::zero();\n  " + SH(1) + "\n  __syncthreads();\n  " + SH(2) + "\n"),
        (H, "  __syncthreads();\n  if (a.heads_out && lead) {",
            "  " + SH(3) + "\n  __syncthreads();\n  " + SH(4) + "\n  if (a.heads_out && lead) {"),
        (H, "  __syncthreads();\n  // ---- phase 3: dz",
            "  " + SH(5) + "\n  __syncthreads();\n  " + SH(6) + "\n  // ---- phase 3: dz"),
        (H, "  // ---- phase 4: dWh partial = dH^T . h over this group's frames (k = frame) ----",
            "  " + SH(7) + "\n  if " + CH + ' { printf("HEAD :"); for (int q = 1; q < 8; ++q) printf(" %lld", st[q] - st[0]); printf("\\n"); }\n  // ---- phase 4: dWh partial = dH^T . h over this group\'s frames (k = frame) ----'),
    ],
}
