# group A gather variants of the two-group fp32 conv12 body, with the PP stamps: wave priority
# raised over the gather, loads batched 4 pixel rows deep, both
import os, runpy
base = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ppstamps32.py"))["VARIANTS"]["ppst"]
C = "conv1.h"
PRIO = [(C, "        gload(0, zt[0], mk[0]);\n", "        __builtin_amdgcn_s_setprio(2);\n        gload(0, zt[0], mk[0]);\n"),
        (C, '        // half 1 reads back the partial sums this wave stored (LDS order per wave)\n        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");\n',
            '        // half 1 reads back the partial sums this wave stored (LDS order per wave)\n        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");\n        __builtin_amdgcn_s_setprio(0);\n')]
B4 = [(C, "        f32x4 zt[2][3];\n        uint32_t mk[2];\n", "        f32x4 zt[4][3];\n        uint32_t mk[4];\n"),
      (C, "        gload(0, zt[0], mk[0]);\n#pragma unroll\n        for (int qy = 0; qy < 8; ++qy) {\n          if (qy + 1 < 8) gload(qy + 1, zt[(qy + 1) & 1], mk[(qy + 1) & 1]);\n",
          "#pragma unroll\n        for (int qy = 0; qy < 8; ++qy) {\n          if ((qy & 3) == 0)\n            for (int u = 0; u < 4; ++u) gload(qy + u, zt[u], mk[u]);\n"),
      (C, "            sum += zt[qy & 1][0];\n            sum += zt[qy & 1][1];\n            v = sum;", "            sum += zt[qy & 3][0];\n            sum += zt[qy & 3][1];\n            v = sum;"),
      (C, "            f32x4 sum = zt[qy & 1][2];\n            sum += zt[qy & 1][0];\n            sum += zt[qy & 1][1];\n            const uint32_t m = pv ? mk[qy & 1] : 0u;",
          "            f32x4 sum = zt[qy & 3][2];\n            sum += zt[qy & 3][0];\n            sum += zt[qy & 3][1];\n            const uint32_t m = pv ? mk[qy & 3] : 0u;")]
VARIANTS = {
    "pg_base": base,
    "pg_prio": base + PRIO,
    "pg_b4": base + B4,
    "pg_b4prio": base + PRIO + B4,
}
