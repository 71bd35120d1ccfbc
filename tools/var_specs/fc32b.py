# round 2 of the fp32 FC / weight-gradient configuration sweep (tools/var_specs/fc32.py)
import os, runpy
_b = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "fc32.py"))
fcf, sp, H, FCS = _b["fcf"], _b["sp"], _b["H"], _b["FCS"]


def fcs(t):
    return (H, FCS, f"  h->spfc = plan_split(N, (FLAT / 256) * (HID / 64), sizeof(float) == 4 ? {t} : 96);")


VARIANTS = {
    "base": [],
    "k256": [fcf(32, 32, 256, 2, 2)],
    "fcs256": [fcs(256)],
    "fcs384": [fcs(384)],
    "sp192": [sp(192, 192)],
    "sp128_256": [sp(128, 256)],
    "sp256_128": [sp(256, 128)],
}
