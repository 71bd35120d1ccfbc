// hostpool.h — a small host thread pool for the staging ring's host-side collate
// (impala_stage_rows): B trajectories scattered in host memory are copied into the slot's
// page-locked block by several threads at once, since one thread's memcpy moves the 15.7 MB of
// a C2 batch in ~1 ms (below PCIe's 0.3 ms for the same bytes).  Host code only.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace impala_host {

// memcpy with streaming (non-temporal) 16-byte stores: the destination is a page-locked block
// the copy engine reads next, so the stores skip the read-for-ownership of a cached store and
// leave the caches to the sources.  Falls back to memcpy when dst / n are not 16-byte aligned.
inline void copy_stream(char* dst, const char* src, size_t n) {
#ifndef __HIP_DEVICE_COMPILE__
  typedef long long v2 __attribute__((vector_size(16)));
  if ((((uintptr_t)dst) | n) & 15) {
    std::memcpy(dst, src, n);
    return;
  }
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    v2 a, b, c, d;
    __builtin_memcpy(&a, src + i, 16);
    __builtin_memcpy(&b, src + i + 16, 16);
    __builtin_memcpy(&c, src + i + 32, 16);
    __builtin_memcpy(&d, src + i + 48, 16);
    __builtin_nontemporal_store(a, (v2*)(dst + i));
    __builtin_nontemporal_store(b, (v2*)(dst + i + 16));
    __builtin_nontemporal_store(c, (v2*)(dst + i + 32));
    __builtin_nontemporal_store(d, (v2*)(dst + i + 48));
  }
  for (; i < n; i += 16) {
    v2 a;
    __builtin_memcpy(&a, src + i, 16);
    __builtin_nontemporal_store(a, (v2*)(dst + i));
  }
  __builtin_ia32_sfence();  // order the streaming stores before the pool's join
#endif
}

class HostPool {
 public:
  explicit HostPool(int nthreads) {
    for (int i = 0; i < nthreads; ++i) th_.emplace_back([this] { worker(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size() + 1; }

  // fn(0 .. ntasks-1), spread over the workers and the calling thread; returns when every task
  // has run.  Calls are serialised by the caller (one staging call at a time per handle).
  void run(int ntasks, const std::function<void(int)>& fn) {
    if (ntasks <= 0) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      ntasks_ = ntasks;
      next_.store(0);
      busy_ = (int)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void drain() {
    for (int i = next_.fetch_add(1); i < ntasks_; i = next_.fetch_add(1)) (*fn_)(i);
  }
  void worker() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      drain();
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--busy_ == 0) done_.notify_one();
      }
    }
  }

  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* fn_ = nullptr;
  int ntasks_ = 0, busy_ = 0;
  std::atomic<int> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace impala_host
