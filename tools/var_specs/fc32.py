# fp32 FC forward tile shapes and weight-gradient split counts (impala.hip launch sites)
H = "impala.hip"
FCF = '''    if (int r = klaunch(h, K_FC_FWD, "fc_fwd", gemm_tile<T, 32, 32, BK(256), 2, 2, FcFwd<T>>,
                        dim3(persist_grid(h, (long)cdiv(n, 32) * (HID / 32))), dim3(256), st, op,
                        HID / 32))
      return r;'''


def fcf(br, bc, bk, wr, wc):
    return (H, FCF, f'''    if constexpr (sizeof(T) == 4) {{
      if (int r = klaunch(h, K_FC_FWD, "fc_fwd", gemm_tile<T, {br}, {bc}, {bk}, {wr}, {wc}, FcFwd<T>>,
                          dim3(persist_grid(h, (long)cdiv(n, {bc}) * (HID / {br}))), dim3(256), st, op,
                          HID / {br}))
        return r;
    }} else {{
''' + FCF + "\n    }")


SP = "  h->sp3 = plan_split((long)N * P3, K3 / 64, 256);\n  h->sp2 = plan_split((long)N * P2, K2 / 128, 256);"


def sp(t3, t2):
    return (H, SP, f"  h->sp3 = plan_split((long)N * P3, K3 / 64, {t3});\n  h->sp2 = plan_split((long)N * P2, K2 / 128, {t2});")


FCS = "  h->spfc = plan_split(N, (FLAT / 256) * (HID / 64), 96);"
VARIANTS = {
    "base": [],
    "f64x32": [fcf(64, 32, 64, 2, 2)],
    "f32x64": [fcf(32, 64, 64, 2, 2)],
    "f64x64": [fcf(64, 64, 64, 2, 2)],
    "f16x64": [fcf(16, 64, 64, 1, 4)],
    "f32x32k128": [fcf(32, 32, 128, 2, 2)],
    "sp384": [sp(384, 384)],
    "sp512": [sp(512, 512)],
    "fcs192": [(H, FCS, "  h->spfc = plan_split(N, (FLAT / 256) * (HID / 64), 192);")],
}
