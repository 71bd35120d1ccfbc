# head_step: which DPP/permlane replacement costs VGPRs (144 -> 246)
SD_V = ("head.h", "const float v_n = shift_down1(v);", "const float v_n = __shfl_down(v, 1, 64);")
SD_T = ("head.h", "const float tgt_n = shift_down1(tgt);", "const float tgt_n = __shfl_down(tgt, 1, 64);")
BIAS = ("head.h", "b = xor32_sum(xor16_sum(b));", "b += __shfl_xor(b, 16, 64);\n      b += __shfl_xor(b, 32, 64);")
VARIANTS = {
    "h_noshift": [SD_V, SD_T],
    "h_nobias": [BIAS],
    "h_none": [SD_V, SD_T, BIAS],
}
