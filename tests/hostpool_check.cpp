// CPU check of impala_amd/csrc/hostpool.h (tests/test_hostpool.py): the thread pool runs every
// task exactly once per call, copy_stream copies exactly, and the staging thread runs jobs in
// order, waits per slot and reports a failed job's status once.
#include "../impala_amd/csrc/hostpool.h"

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                    \
    }                                                              \
  } while (0)

int main() {
  using namespace impala_host;
  // pool: 1000 calls of 257 tasks on 3 workers + the caller
  {
    HostPool pool(3, local_node_cpus());
    std::vector<std::atomic<int>> hits(257);
    for (int rep = 0; rep < 1000; ++rep)
      pool.run(257, [&](int i) { hits[i].fetch_add(1); });
    for (auto& h : hits) CHECK(h.load() == 1000);
  }
  // streaming copy: aligned and unaligned sizes / destinations
  {
    std::vector<char> src(70001), dst(70016 + 16);
    for (size_t i = 0; i < src.size(); ++i) src[i] = (char)(i * 131 + 7);
    for (size_t n : {0ul, 16ul, 48ul, 64ul, 65536ul, 70000ul, 70001ul})
      for (size_t off : {0ul, 16ul, 3ul}) {
        std::fill(dst.begin(), dst.end(), 0);
        copy_stream(dst.data() + off + (16 - ((uintptr_t)dst.data() & 15)) % 16, src.data(), n);
        const char* d = dst.data() + off + (16 - ((uintptr_t)dst.data() & 15)) % 16;
        for (size_t i = 0; i < n; ++i) CHECK(d[i] == src[i]);
      }
  }
  // stager: in-order jobs, per-slot waits, one failure reported once
  {
    Stager st;
    std::vector<int> order;
    std::mutex mu;
    for (int j = 0; j < 40; ++j)
      st.submit(j % 3, [&, j](std::string& msg) {
        std::lock_guard<std::mutex> lk(mu);
        order.push_back(j);
        if (j == 7) {
          msg = "job 7";
          return 42;
        }
        return 0;
      });
    std::string m;
    CHECK(st.wait(1, m) == 42 && m == "job 7");  // slot 1 ran job 7
    m.clear();
    CHECK(st.wait(-1, m) == 0 && m.empty());      // reported once
    CHECK(order.size() == 40);
    for (int j = 0; j < 40; ++j) CHECK(order[j] == j);
  }
  std::printf("hostpool ok\n");
  return 0;
}
