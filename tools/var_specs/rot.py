C = "conv1.h"
L = "lnc3.h"
OLD = "const int e = (int)threadIdx.x + i * NT"
NEW = "const int e = (int)threadIdx.x + ((i + ((int)(blockIdx.x >> 3) % NPT)) % NPT) * NT"
def rep(f, n):
    return [(f, OLD, NEW)] * n
VARIANTS = {"base": [], "rot": [("conv1.h", OLD, NEW)]}
