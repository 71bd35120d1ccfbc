H = "impala.hip"
L = "      while (sg < 16 && sg * 4 < S) sg <<= 1;  // ~4+ loads per thread, <= 16 groups"
VARIANTS = {
    "base": [],
    "sg8": [(H, L, L.replace("sg < 16", "sg < 8"))],
    "sg4": [(H, L, L.replace("sg < 16", "sg < 4"))],
    "sg2": [(H, L, L.replace("sg < 16", "sg < 2"))],
}
