# Slab reduction split groups (impala.hip reduce plan): the cap on split groups per workgroup
# raised 16 -> 32, with 8 split loads per thread, so the 256-split slabs (conv1, LayerNorm)
# load in one round of 8 instead of two (32 columns of 4 floats per workgroup; a 32-way combine).
H = "impala.hip"
VARIANTS = {
    "redsg32": [(H, "      while (sg < 16 && sg * lpt < S) sg <<= 1;  // ~lpt+ loads per thread, <= 16 groups",
                 "      while (sg < 32 && sg * lpt < S) sg <<= 1;  // ~lpt+ loads per thread, <= 32 groups"),
                (H, "    int lpt = 16;", "    int lpt = 8;")],
}
