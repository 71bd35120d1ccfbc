# reduce_grads knock-outs (timing only): no canonical grad stores / no slab loads
K = "kernels.h"
ST = """  for (int i = 0; i < 4; ++i)
    if (ci[i] >= 0) a.grads[ci[i]] = acc[i];
  sq = wave_sum(sq);"""
LD = """    acc = (sg.S + r.SG - 1) / r.SG <= 8 ? sum_splits<8>(p, r.grp, r.SG, sg.S, sg.count)
                                        : sum_splits<16>(p, r.grp, r.SG, sg.S, sg.count);"""
VARIANTS = {
    "red_base": [],
    "red_nostore": [(K, ST, """  for (int i = 0; i < 4; ++i)
    if (ci[i] >= 0 && acc[i] == 12345.f) a.grads[ci[i]] = acc[i];
  sq = wave_sum(sq);""")],
    "red_noload": [(K, LD, """    acc = f32x4{(float)r.v4, 0.f, 0.f, 0.f};""")],
    "red_s1load": [(K, LD, """    acc = *reinterpret_cast<const f32x4*>(p);""")],
}
