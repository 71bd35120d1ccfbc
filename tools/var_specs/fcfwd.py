# FC forward tile shapes (gemm_tile<FcFwd>: rows = 256 hidden units, cols = frames, K = 1024)
H = "impala.hip"
OLD = """    if (int r = klaunch(h, K_FC_FWD, "fc_fwd", gemm_tile<T, 64, 32, BK(256), 2, 2, FcFwd<T>>,
                        dim3(persist_grid(h, (long)cdiv(n, 32) * (HID / 64))), dim3(256), st, op,
                        HID / 64))"""
def V(br, bc, bk, wr, wc):
    return [(H, OLD, f"""    if (int r = klaunch(h, K_FC_FWD, "fc_fwd", gemm_tile<T, {br}, {bc}, BK({bk}), {wr}, {wc}, FcFwd<T>>,
                        dim3(persist_grid(h, (long)cdiv(n, {bc}) * (HID / {br}))), dim3(256), st, op,
                        HID / {br}))""")]
VARIANTS = {
    "f64x32k256": [],
    "f32x32k256": V(32, 32, 256, 2, 2),
    "f32x32k128": V(32, 32, 128, 2, 2),
    "f64x32k128": V(64, 32, 128, 2, 2),
}
