#pragma once

#include "common.h"

namespace sfa {

struct KfpnOut {
  float* ptr[SFA_MAX_HEADS];  // NCHW (B, ch[j], h, w) per head, forward order
  int ch[SFA_MAX_HEADS];
  int off[SFA_MAX_HEADS];     // first planar channel of head j
  int num_heads;
  int total_ch;
};

// amax (nullable): per-frame max |y| words (conv.h, fp16x3 input scale)
int launch_nchw3_to_nhwc4(const float* x, float* y, int B, int H, int W, bool flip, unsigned* amax,
                          hipStream_t st);
int launch_amax_nhwc4(const float* x, int B, int H, int W, unsigned* amax, hipStream_t st);
int launch_maxpool3s2(const float* x, float* y, int B, int H, int W, int C, hipStream_t st);
int launch_upsample2x(const float* x, float* y, int B, int H, int W, int C, hipStream_t st);
int launch_kfpn(const float* L0, const float* L1, const float* L2, const KfpnOut& o, int B, int h,
                int w, hipStream_t st);
int launch_sigmoid_clamp(float* x, long long n, hipStream_t st);
// Zero `bytes` (a multiple of 4, 4-B aligned) of device memory with a kernel instead of
// hipMemsetAsync: on this ROCm a memset captured into a single-branch HIP graph is replayed from a
// kernel-argument slot that later launches reuse, so the replayed node zeroes whatever that slot
// then points at (tools/debug/graph_repro.py); kernel nodes keep their own arguments.
int launch_zero_words(void* p, size_t bytes, hipStream_t st);

}  // namespace sfa
