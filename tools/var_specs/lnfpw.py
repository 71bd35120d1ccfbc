H = "impala.hip"
def fpw(n):
    return [(H, "  int n_ln_wg = 0, ln_fpw = 4,", f"  int n_ln_wg = 0, ln_fpw = {n},")]
VARIANTS = {"fpw4": [], "fpw2": fpw(2), "fpw1": fpw(1)}
