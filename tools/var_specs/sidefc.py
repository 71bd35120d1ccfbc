# the FC weight gradient (80 workgroups) on a side stream, beside FC dgrad + LayerNorm/conv3 dgrad
F = "impala.hip"
E = [
    (F, "  bool use_side = true;", "  bool use_side = true;\n  bool side_fc = false;"),
    (F, """  const char* side = std::getenv("IMPALA_SIDE_STREAM");
  if (!side || side[0] != '1') {
    h->use_side = false;""", """  const char* side = std::getenv("IMPALA_SIDE_STREAM");
  h->side_fc = true;
  if (!side || side[0] != '1') {
    h->use_side = false;
    if (hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking) != hipSuccess) h->side_fc = false;
    for (int i = 0; i < 4; ++i)
      if (hipEventCreateWithFlags(&h->ev_fork[i], hipEventDisableTiming) != hipSuccess) h->side_fc = false;
    if (hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) != hipSuccess) h->side_fc = false;"""),
    (F, """  if (int r = fork(1)) return r;  // dz ready
  {
    FcWgrad<T> op{};""", """  if (int r = fork(1)) return r;  // dz ready
  if (sfc) {
    CK(hipEventRecord(h->ev_fork[1], st));
    CK(hipStreamWaitEvent(h->side, h->ev_fork[1], 0));
  }
  {
    hipStream_t ss = sfc ? h->side : (h->use_side ? h->side : st);
    FcWgrad<T> op{};"""),
    (F, """  if (h->red_mode == 0) {
    if (h->use_side) {  // join""", """  if (sfc) {
    CK(hipEventRecord(h->ev_join, h->side));
    CK(hipStreamWaitEvent(st, h->ev_join, 0));
  }
  if (h->red_mode == 0) {
    if (h->use_side) {  // join"""),
]
E.append((F, "  if (part == 1 || part == 4) goto part1;", "  const bool sfc = h->side_fc && part == -1;\n  if (part == 1 || part == 4) goto part1;"))
VARIANTS = {"base": [], "sidefc": E}
