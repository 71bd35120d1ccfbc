K = "kernels.h"
H = "impala.hip"
SEQ = (K, '''  // fixed-order tree over the SG split groups
  for (int half = SG >> 1; half > 0; half >>= 1) {
    if (grp < half) {
      acc += part[(grp + half) * cols + col];
      part[threadIdx.x] = acc;
    }
    __syncthreads();
  }
  float sq = 0.f;
  if (grp == 0 && in) {''', '''  float sq = 0.f;
  if (grp == 0 && in) {
    for (int g2 = 1; g2 < SG; ++g2) acc += part[g2 * cols + col];''')
def cap(n):
    return (H, "      while (sg < 64 && sg * 4 <= S) sg <<= 1;", f"      while (sg < {n} && sg * 4 <= S) sg <<= 1;")
VARIANTS = {"seq16": [SEQ, cap(16)], "tree16": [cap(16)], "tree32": [cap(32)], "tree64": []}
