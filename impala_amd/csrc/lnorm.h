// LayerNorm of one frame's conv3 output (models/common.py:120-126: ReLU, then LayerNorm over
// the 1024 = 16 pixels x 64 channels features), shared by the tiled conv3 GEMM epilogue and the
// fused forward trunk so both produce bit-identical act3 / y / stats.
#pragma once
#include "common.h"
#include "net.h"

// The per-lane constants of the epilogue (lane owns features 16*lane .. 16*lane+15: pixel
// lane/4, channels 16*(lane%4) ..): conv3 bias, LayerNorm gamma / beta (p*64+c order).
struct LnLane {
  float b[16], g[16], e[16];
};
DEV LnLane ln_lane_consts(int lane, const float* b3, const float* gam, const float* bet) {
  LnLane c;
  const int c0 = (lane & 3) * 16;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    c.b[i] = b3[c0 + i];
    c.g[i] = gam[lane * 16 + i];
    c.e[i] = bet[lane * 16 + i];
  }
  return c;
}

// One wavefront per frame.  et: fp32 conv3 accumulators of the frame, [16 px][ldt]
// channels-contiguous.  Writes act3 = relu(acc + b3), y = LN(act3) and (mean, rstd).
// Y_SC1 (bf16): y is stored write-through (8-byte agent-scope atomic stores = sc1), the payload
// form another workgroup of the same launch may read after a flag (fwd_chain_kernel).
template <typename T, bool Y_SC1 = false>
DEV void ln_frame_epilogue(const float* et, int ldt, int frame, int lane, const LnLane& k,
                           T* act3, T* y, float* stats) {
  using namespace net;
  const int p = lane >> 2, c0 = (lane & 3) * 16;
  const float* src = et + p * ldt + c0;
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = fmaxf(src[i] + k.b[i], 0.f);
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) sum += v[i];
  const float mean = wave_sum(sum) * (1.f / FLAT);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) q += (v[i] - mean) * (v[i] - mean);
  const float rstd = 1.f / sqrtf(wave_sum(q) * (1.f / FLAT) + LN_EPS);
  const size_t o = (size_t)frame * FLAT + lane * 16, oy = (size_t)frame * YLD + lane * 16;
#pragma unroll
  for (int i = 0; i < 16; i += 4) {
    float yy[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      yy[q] = (v[i + q] - mean) * rstd * k.g[i + q] + k.e[i + q];
    store4(act3 + o + i, v + i);
    if constexpr (Y_SC1 && sizeof(T) == 2) {
      const unsigned long long w = (unsigned long long)(unsigned)pack_bf16x2(yy[0], yy[1]) |
                                   ((unsigned long long)(unsigned)pack_bf16x2(yy[2], yy[3]) << 32);
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(y + oy + i), w, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    } else {
      store4(y + oy + i, yy);
    }
  }
  if (lane == 0) {
    stats[2 * frame] = mean;
    stats[2 * frame + 1] = rstd;
  }
}

// M frames of one wavefront at once (the fp32 forward tail: 5 frames on 4 waves), each with
// exactly the arithmetic of ln_frame_epilogue; the M independent reduction chains interleave.
template <typename T, int M>
DEV void ln_frames_epilogue(const float* et, int fstride, int ldt, const int (&frame)[M], int lane,
                            const LnLane& k, T* act3, T* y, float* stats) {
  using namespace net;
  const int p = lane >> 2, c0 = (lane & 3) * 16;
  float v[M][16], mean[M], rstd[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const float* src = et + m * fstride + p * ldt + c0;
#pragma unroll
    for (int i = 0; i < 16; ++i) v[m][i] = fmaxf(src[i] + k.b[i], 0.f);
  }
  float sum[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    sum[m] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) sum[m] += v[m][i];
  }
#pragma unroll
  for (int m = 0; m < M; ++m) mean[m] = wave_sum(sum[m]) * (1.f / FLAT);
  float q[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    q[m] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) q[m] += (v[m][i] - mean[m]) * (v[m][i] - mean[m]);
  }
#pragma unroll
  for (int m = 0; m < M; ++m) rstd[m] = 1.f / sqrtf(wave_sum(q[m]) * (1.f / FLAT) + LN_EPS);
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const size_t o = (size_t)frame[m] * FLAT + lane * 16, oy = (size_t)frame[m] * YLD + lane * 16;
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
      float yy[4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        yy[c] = (v[m][i + c] - mean[m]) * rstd[m] * k.g[i + c] + k.e[i + c];
      store4(act3 + o + i, v[m] + i);
      store4(y + oy + i, yy);
    }
    if (lane == 0) {
      stats[2 * frame[m]] = mean[m];
      stats[2 * frame[m] + 1] = rstd[m];
    }
  }
}

