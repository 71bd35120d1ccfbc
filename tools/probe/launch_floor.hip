// What a dependent kernel boundary costs on this box (DESIGN.md §7 "every launch costs 4-5 us").
// Back-to-back launches of trivial kernels on one stream, timed three ways:
//   * hipEvents around 200 launches (per-launch period);
//   * device stamps (s_memrealtime, 100 MHz): every workgroup of every launch stores its start and
//     end into its own slot (plain vector stores: same-address atomics from 1024 workgroups
//     serialise at one L2 channel and cost ~20 us themselves); the host takes the first start and
//     the last end per launch, so start[i+1] - end[i] is the idle gap between dependent kernels
//     as the device sees it;
//   * the same 200 launches captured in a hipGraph.
// Shapes: 1 workgroup; 1024 workgroups of 256 threads; 1024 workgroups with a 1 KB kernel
// argument block; 600 workgroups that each load + store one float4 per thread (adam-like).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/launch_floor tools/probe/launch_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

struct Big { float v[256]; };

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

constexpr int WGMAX = 1024;  // stamp slots per launch: [2 * WGMAX] = {start, end} per workgroup
__device__ __forceinline__ void stamp_begin(unsigned long long* s) {
  if (threadIdx.x == 0) s[2 * blockIdx.x] = now();
}
__device__ __forceinline__ void stamp_end(unsigned long long* s) {
  __syncthreads();
  if (threadIdx.x == 0) s[2 * blockIdx.x + 1] = now();
}

__global__ void k_empty(unsigned long long* s) { stamp_begin(s); stamp_end(s); }
__global__ void k_bigarg(unsigned long long* s, const Big b, float* out) {
  stamp_begin(s);
  if (b.v[threadIdx.x & 255] == 12345.f) out[0] = 1.f;  // never true: keeps the argument live
  stamp_end(s);
}
__global__ void k_rw(unsigned long long* s, float4* x, int n) {
  stamp_begin(s);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { float4 v = x[i]; v.x += 1.f; x[i] = v; }
  stamp_end(s);
}


int main(int argc, char** argv) {
  const int L = 200;
  unsigned long long* st;
  const size_t NS = (size_t)2 * WGMAX * L;
  CK(hipMalloc(&st, sizeof(unsigned long long) * NS));
  float4* x;
  const int nx = 600 * 256;
  CK(hipMalloc(&x, sizeof(float4) * nx));
  CK(hipMemset(x, 0, sizeof(float4) * nx));
  float* out;
  CK(hipMalloc(&out, 4));
  Big big{};
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<unsigned long long> hs(NS), h(2 * L);
  const int nwg[4] = {1, 1024, 1024, 600};

  auto launch = [&](int kind, int i) {
    unsigned long long* p = st + (size_t)2 * WGMAX * i;
    switch (kind) {
      case 0: k_empty<<<1, 64, 0, s>>>(p); break;
      case 1: k_empty<<<1024, 256, 0, s>>>(p); break;
      case 2: k_bigarg<<<1024, 256, 0, s>>>(p, big, out); break;
      case 3: k_rw<<<600, 256, 0, s>>>(p, x, nx); break;
    }
  };
  const char* names[4] = {"empty 1x64", "empty 1024x256", "1KB arg 1024x256", "rw float4 600x256"};
  for (int kind = 0; kind < 4; ++kind) {
    for (int mode = 0; mode < 2; ++mode) {  // 0: stream launches, 1: hipGraph replay
      hipGraphExec_t ge = nullptr;
      hipGraph_t g = nullptr;
      if (mode == 1) {
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < L; ++i) launch(kind, i);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      }
      float best = 1e30f;
      double gap_med = 0, dur_med = 0, per_dev = 0;
      for (int rep = 0; rep < 5; ++rep) {
        // a busy kernel first, so the timed launches queue up behind it
        for (int i = 0; i < 20; ++i) launch(kind, 0);
        CK(hipEventRecord(e0, s));
        if (mode == 0)
          for (int i = 0; i < L; ++i) launch(kind, i);
        else
          CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) {
          best = ms;
          CK(hipMemcpy(hs.data(), st, sizeof(unsigned long long) * NS, hipMemcpyDeviceToHost));
          for (int i = 0; i < L; ++i) {
            const unsigned long long* q = hs.data() + (size_t)2 * WGMAX * i;
            unsigned long long b = ~0ull, e = 0;
            for (int w = 0; w < nwg[kind]; ++w) { b = std::min(b, q[2 * w]); e = std::max(e, q[2 * w + 1]); }
            h[2 * i] = b;
            h[2 * i + 1] = e;
          }
          std::vector<double> gap, dur;
          for (int i = 10; i + 1 < L; ++i) {
            gap.push_back((double)(h[2 * (i + 1)] - h[2 * i + 1]) * 10.0);  // ns
            dur.push_back((double)(h[2 * i + 1] - h[2 * i]) * 10.0);
          }
          std::sort(gap.begin(), gap.end());
          std::sort(dur.begin(), dur.end());
          gap_med = gap[gap.size() / 2];
          dur_med = dur[dur.size() / 2];
          per_dev = (double)(h[2 * (L - 1)] - h[2 * 10]) * 10.0 / (L - 11);
        }
      }
      std::printf("%-20s %-6s events %.3f us/launch | device: period %.3f us, busy %.3f us, "
                  "gap %.3f us (medians)\n",
                  names[kind], mode ? "graph" : "stream", best * 1e3 / L, per_dev * 1e-3,
                  dur_med * 1e-3, gap_med * 1e-3);
      if (ge) CK(hipGraphExecDestroy(ge));
      if (g) CK(hipGraphDestroy(g));
    }
  }
  CK(hipStreamSynchronize(s));
  return 0;
}
