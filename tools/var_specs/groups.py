C = "conv1.h"
H = "impala.hip"
FWD_G1 = [(C, "template <typename T> constexpr int c12f_groups() { return sizeof(T) == 2 ? 2 : 1; }",
              "template <typename T> constexpr int c12f_groups() { return 1; }"),
          (H, "    const int fpw = std::max(1, cdiv(n, h->n_cu));", "    const int fpw = std::max(1, cdiv(n, 2 * h->n_cu));")]
BWD_G1 = [(C, "template <typename T> constexpr int c12_groups() { return sizeof(T) == 2 ? 2 : 1; }",
              "template <typename T> constexpr int c12_groups() { return 1; }"),
          (H, "  h->c1_fpw = std::max(1, cdiv(N, h->n_cu));", "  h->c1_fpw = std::max(1, cdiv(N, 2 * h->n_cu));")]
VARIANTS = {"base": [], "fwd_g1": FWD_G1, "bwd_g1": BWD_G1}
