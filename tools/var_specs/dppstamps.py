import runpy, os
D = os.path.dirname(os.path.abspath(__file__))
ST = runpy.run_path(os.path.join(D, "headstamps.py"))["VARIANTS"]["hstamps"]
SD_V = ("head.h", "const float v_n = shift_down1(v);", "const float v_n = __shfl_down(v, 1, 64);")
SD_T = ("head.h", "const float tgt_n = shift_down1(tgt);", "const float tgt_n = __shfl_down(tgt, 1, 64);")
WS = ("head.h", "s0 = wave_sum(s0); s1 = wave_sum(s1);\n    const float s2 = wave_sum(H), s3 = wave_sum(kld), s4 = wave_sum(rho);",
      "s0 = wave_sum_x(s0); s1 = wave_sum_x(s1);\n    const float s2 = wave_sum_x(H), s3 = wave_sum_x(kld), s4 = wave_sum_x(rho);")
WSX = ("common.h", "DEV float wave_max(", "DEV float wave_sum_x(float v) {\n#pragma unroll\n  for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);\n  return v;\n}\nDEV float wave_max(")
VARIANTS = {
    "s_dpp": ST,
    "s_noshift": ST + [SD_V, SD_T],
    "s_xsum": ST + [WS, WSX],
    "s_both": ST + [SD_V, SD_T, WS, WSX],
}
