// hostpool.h — a small host thread pool for the staging ring's host-side collate
// (impala_stage_rows): B trajectories scattered in host memory are copied into the slot's
// page-locked block by several threads at once, since one thread's memcpy moves the 15.7 MB of
// a C2 batch in ~1 ms (below PCIe's 0.3 ms for the same bytes).  Host code only.
#pragma once

#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <string>
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

// The CPUs of a NUMA node, within the process's affinity set (empty when the topology cannot be
// read): where the staging threads run (impala_stage_rows_async; impala.hip stage_cpus).
// node < 0: the node of the CPU the calling thread runs on
inline std::vector<int> local_node_cpus(int node = -1) {
  std::vector<int> out;
#ifndef __HIP_DEVICE_COMPILE__
  if (node < 0) {
    const int cpu = sched_getcpu();
    if (cpu < 0) return out;
    for (int n = 0; n < 64 && node < 0; ++n) {
      char path[96];
      std::snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/node%d", cpu, n);
      if (access(path, F_OK) == 0) node = n;
    }
  }
  if (node < 0) return out;
  char path[96];
  std::snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = std::fopen(path, "r");
  if (!f) return out;
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) {
    std::fclose(f);
    return out;
  }
  int a = 0, b = 0;
  char sep = 0;
  while (std::fscanf(f, "%d", &a) == 1) {
    b = a;
    if (std::fscanf(f, "%c", &sep) == 1 && sep == '-') {
      if (std::fscanf(f, "%d", &b) != 1) break;
      if (std::fscanf(f, "%c", &sep) != 1) sep = 0;
    }
    for (int c = a; c <= b; ++c)
      if (c < CPU_SETSIZE && CPU_ISSET(c, &allowed)) out.push_back(c);
    if (sep != ',') break;
  }
  std::fclose(f);
#endif
  return out;
}

// pin the calling thread to `cpus` (no-op when empty)
inline void pin_to(const std::vector<int>& cpus) {
#ifndef __HIP_DEVICE_COMPILE__
  if (cpus.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus) CPU_SET(c, &set);
  (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
#endif
}

class HostPool {
 public:
  // nthreads workers, kept on `cpus` (the creating thread's NUMA node, local_node_cpus) when
  // non-empty
  explicit HostPool(int nthreads, std::vector<int> cpus = {}) {
    for (int i = 0; i < nthreads; ++i) th_.emplace_back([this, cpus] {
      pin_to(cpus);
      worker();
    });
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

// One background thread that runs staging jobs in order (impala_stage_rows_async): the caller
// hands over a job and returns at once; `pending(slot)` jobs per slot are waited for by the
// calls that use the slot.  A job's status and error text are kept for the next waiter.
class Stager {
 public:
  explicit Stager(std::vector<int> cpus = {}) : th_([this, cpus] {
    pin_to(cpus);
    loop();
  }) {}
  ~Stager() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void submit(int slot, std::function<int(std::string&)> job) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      ++pending_[slot];
      q_.push_back({slot, std::move(job)});
    }
    cv_.notify_all();
  }
  // wait until `slot` (every slot when < 0) has no job queued or running; -> the first failed
  // job's status since the last wait (0 = ok), its message in `msg`
  int wait(int slot, std::string& msg) {
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] {
      if (slot >= 0) return pending_[slot] == 0;
      for (int p : pending_)
        if (p) return false;
      return true;
    });
    int r = 0;
    for (int i = 0; i < kSlots; ++i)
      if ((slot < 0 || i == slot) && err_[i]) {
        if (!r) {
          r = err_[i];
          msg = msg_[i];
        }
        err_[i] = 0;
      }
    return r;
  }
  static constexpr int kSlots = 8;

 private:
  struct Job {
    int slot;
    std::function<int(std::string&)> fn;
  };
  void loop() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;  // stop, and nothing left to run
        j = std::move(q_.front());
        q_.pop_front();
      }
      std::string m;
      const int r = j.fn(m);
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (r && !err_[j.slot]) {
          err_[j.slot] = r;
          msg_[j.slot] = m;
        }
        --pending_[j.slot];
      }
      done_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::deque<Job> q_;
  int pending_[kSlots] = {};
  int err_[kSlots] = {};
  std::string msg_[kSlots];
  bool stop_ = false;
  std::thread th_;
};

}  // namespace impala_host
