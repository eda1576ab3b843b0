// Round-5 diagnostic: s_memtime stamps of the fused heads kernel (tools/experiments/r05/conv_r3_stamp.h,
// generated from the product conv_r3 body) on the three KFPN levels at bs 16 (L0: 76^2 x 256, L1: 152^2 x 128,
// L2: 152^2 x 64), written to gpurun_out/hstamps_<name>.bin: int32 header {nblocks, waves per block, record
// words, K-tiles}, then uint64 records (tools/head_stamp_summary.py).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -pthread tools/headstampbench.hip -o tools/headstampbench
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>
#include <chrono>
#include <thread>

#include "../lidar-image_object-detection_-fpn_resnet-yolov8_amd/csrc/conv_h3_kernel.h"
#include "../lidar-image_object-detection_-fpn_resnet-yolov8_amd/csrc/conv_r3_kernel.h"
#include "experiments/r05/conv_r3_stamp.h"

namespace sfa {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fprintf(stderr, "\n");
}
}  // namespace sfa

using namespace sfa;

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

static float* dev_random(size_t n, unsigned seed, float scale) {
  std::vector<float> h(n);
  unsigned s = seed * 2654435761u + 12345u;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    h[i] = scale * ((float)(s >> 8) / 16777216.0f - 0.5f);
  }
  float* d;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

// [N][Kpad] f32 (device) -> fp16x3 terms [2][N][Kpad] of w * 2^(13 - e[n]) and winv[n]
static void split_weights_h3(const float* w, int N, int Kpad, uint16_t** wh, float** winv) {
  const size_t n = (size_t)N * Kpad;
  std::vector<float> hw(n), inv(N);
  CK(hipMemcpy(hw.data(), w, n * 4, hipMemcpyDeviceToHost));
  std::vector<_Float16> hs(2 * n);
  for (int o = 0; o < N; ++o) {
    float mx = 0.f;
    for (int k = 0; k < Kpad; ++k) mx = std::max(mx, std::fabs(hw[(size_t)o * Kpad + k]));
    int e = 0;
    if (mx > 0.f) (void)std::frexp(mx, &e), e -= 1;  // mx in [2^e, 2^(e+1))
    const float sc = std::ldexp(1.f, 13 - e);
    inv[o] = std::ldexp(1.f, e - 13);
    for (int k = 0; k < Kpad; ++k) {
      const size_t i = (size_t)o * Kpad + k;
      const float x = hw[i] * sc;
      const _Float16 hi = (_Float16)x;
      hs[i] = hi;
      hs[n + i] = (_Float16)(x - (float)hi);
    }
  }
  CK(hipMalloc(wh, hs.size() * 2));
  CK(hipMemcpy(*wh, hs.data(), hs.size() * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(winv, N * 4));
  CK(hipMemcpy(*winv, inv.data(), N * 4, hipMemcpyHostToDevice));
}



int main(int argc, char** argv) {
  constexpr int R3_HEAD_STAG = 256 | 2048 | 4 | 4096 | 8192 | 16384 | 65536 | 524288 | 1048576 | 2097152;  // conv.hip (experiment bit)
  struct Sh { const char* name; int H, C; };
  const Sh shapes[] = {{"L0", 76, 256}, {"L1", 152, 128}, {"L2", 152, 64}};
  const int hch[5] = {3, 2, 2, 1, 3}, nhead = 5, N = 320;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (const Sh& sh : shapes) {
    if (argc > 1 && !strstr(sh.name, argv[1])) continue;
    const int B = 16, M = B * sh.H * sh.H, K = 9 * sh.C;
    float* x = dev_random((size_t)M * sh.C, 1, 1.0f);
    std::vector<unsigned> words((size_t)B * SFA_AMAX_WORDS, 0u);
    for (int b = 0; b < B; ++b) { const float mx = 0.5f; memcpy(&words[(size_t)b * SFA_AMAX_WORDS], &mx, 4); }
    unsigned* amax_x;
    CK(hipMalloc(&amax_x, words.size() * 4));
    CK(hipMemcpy(amax_x, words.data(), words.size() * 4, hipMemcpyHostToDevice));
    float* w = dev_random((size_t)N * K, 2, 2.0f / std::sqrt((float)K));
    float* bias = dev_random(N, 3, 0.2f);
    float* hw1 = dev_random((size_t)nhead * 4 * 64, 4, 0.25f);
    float* hb1 = dev_random((size_t)nhead * 4, 5, 0.2f);
    float* hout;
    CK(hipMalloc(&hout, (size_t)11 * M * 4));
    uint16_t* whp;
    float* winvp;
    split_weights_h3(w, N, K, &whp, &winvp);
    ConvArgs a;
    memset(&a, 0, sizeof a);
    a.nseg = 1;
    make_seg(a.seg[0], x, B, sh.H, sh.H, sh.C, 3, 1, 1);
    a.w = w; a.wh = whp; a.winv = winvp; a.amax_in[0] = amax_x;
    a.bias = bias; a.M = M; a.N = N; a.OH = sh.H; a.OW = sh.H; a.relu = 1; a.Kpad = K;
    a.hw1 = hw1; a.hb1 = hb1; a.hout = hout;
    for (int j = 0, off = 0; j < nhead; ++j) { a.hch[j] = hch[j]; a.hoff[j] = off; off += hch[j]; }
    const int nblocks = (M + 255) / 256, NW = 8;
    unsigned long long* stp;
    CK(hipMalloc(&stp, (size_t)nblocks * NW * HST_REC * 8));
    CK(hipMemset(stp, 0, (size_t)nblocks * NW * HST_REC * 8));
    a.part = reinterpret_cast<float*>(stp);
    a.ksplit = 1;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms = 0.f;
    for (int it = 0; it < 4; ++it) {  // warm (caches, clocks), the last launch's stamps are kept
      CK(hipEventRecord(e0, st));
      const int rc = launch_conv_r3_stamp_cfg<256, 320, 32, EPI_HEAD, 1, 3, R3_HEAD_STAG>(a, st);
      CK(hipEventRecord(e1, st));
      if (rc != SFA_OK) { printf("%s: launch failed\n", sh.name); return 1; }
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    std::vector<unsigned long long> h((size_t)nblocks * NW * HST_REC);
    CK(hipMemcpy(h.data(), stp, h.size() * 8, hipMemcpyDeviceToHost));
    const int nkt = K / 32;
    char fn[256];
    snprintf(fn, sizeof fn, "gpurun_out/hstamps_%s.bin", sh.name);
    FILE* f = fopen(fn, "wb");
    const int hdr[4] = {nblocks, NW, HST_REC, nkt};
    fwrite(hdr, 4, 4, f);
    fwrite(h.data(), 8, h.size(), f);
    fclose(f);
    printf("%s: %d blocks x %d waves, %d K-tiles, last launch %.1f us (stamped) -> %s\n", sh.name, nblocks, NW, nkt,
           ms * 1000.f, fn);
    CK(hipFree(x)); CK(hipFree(amax_x)); CK(hipFree(w)); CK(hipFree(bias)); CK(hipFree(hw1)); CK(hipFree(hb1));
    CK(hipFree(hout)); CK(hipFree(whp)); CK(hipFree(winvp)); CK(hipFree(stp));
  }
  return 0;
}
