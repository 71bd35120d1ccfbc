# per-workgroup span of conv12_fwd_s2d in s_memrealtime (100 MHz) ticks: start, end (every 16th WG)
F = "conv1.h"
VARIANTS = {
    "fspan": [
        (F, "  const int kl = KPL * (lane >> 4);\n  uint4 nv[3];\n  if (f0 + grp < f1) c1_load_frame<T>(x + (size_t)(f0 + grp) * IMG, tid, nv);",
            "  const int kl = KPL * (lane >> 4);\n  const long long t_start = __builtin_amdgcn_s_memrealtime();\n  uint4 nv[3];\n  if (f0 + grp < f1) c1_load_frame<T>(x + (size_t)(f0 + grp) * IMG, tid, nv);\n  "),
        (F, "          store4(act2 + ((size_t)f * P2 + pc) * OC2 + 16 * wave + 4 * (lane >> 4), v);\n        }\n      }\n    }\n  }\n}",
            "          store4(act2 + ((size_t)f * P2 + pc) * OC2 + 16 * wave + 4 * (lane >> 4), v);\n        }\n      }\n    }\n  }\n  " + 'if (blockIdx.x % 16 == 0 && threadIdx.x == 0) printf("SPAN %d %lld %lld\\n", (int)blockIdx.x, t_start, (long long)__builtin_amdgcn_s_memrealtime());\n}'),
    ],
}
