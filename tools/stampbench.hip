// Round-5 diagnostic: per-k-step s_memtime stamps of the strip kernel (tools/experiments/r05/
// conv_h3s_stamp.h) on the layer1 / layer2 / layer4 shapes at bs 16, written to gpurun_out/stamps_<name>.bin:
// int32 header {nblocks, waves per block, record words, k-steps}, then uint64 records.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -pthread tools/stampbench.hip -o tools/stampbench
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

#include "../lidar-image_object-detection_-fpn_resnet-yolov8_amd/csrc/conv_kernel.h"
#include "../lidar-image_object-detection_-fpn_resnet-yolov8_amd/csrc/conv_x6_kernel.h"
#include "../lidar-image_object-detection_-fpn_resnet-yolov8_amd/csrc/conv_h3_kernel.h"
#include "../lidar-image_object-detection_-fpn_resnet-yolov8_amd/csrc/conv_h3s_kernel.h"
#include "../lidar-image_object-detection_-fpn_resnet-yolov8_amd/csrc/conv_r3_kernel.h"
#include "experiments/r05/conv_h3s_stamp.h"

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

static uint16_t bf16_rne(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float bf16_f(uint16_t b) {
  unsigned u = (unsigned)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
// [N][Kpad] f32 (device) -> [3][N][Kpad] bf16 terms (device)
static uint16_t* split_weights(const float* w, size_t n) {
  std::vector<float> hw(n);
  CK(hipMemcpy(hw.data(), w, n * 4, hipMemcpyDeviceToHost));
  std::vector<uint16_t> hs(3 * n);
  for (size_t i = 0; i < n; ++i) {
    float x = hw[i];
    for (int t = 0; t < 3; ++t) {
      const uint16_t b = bf16_rne(x);
      hs[t * n + i] = b;
      x -= bf16_f(b);
    }
  }
  uint16_t* d;
  CK(hipMalloc(&d, hs.size() * 2));
  CK(hipMemcpy(d, hs.data(), hs.size() * 2, hipMemcpyHostToDevice));
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
  struct Sh { const char* name; int H, C, N, BM, WM; bool res; int ks; };
  const Sh shapes[] = {{"layer1", 152, 64, 64, 128, 32, true, 1}, {"layer2", 76, 128, 128, 128, 32, false, 1},
                       {"layer4", 19, 512, 512, 128, 32, false, 2}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  float* part;
  CK(hipMalloc(&part, (size_t)64 << 22));
  for (const Sh& sh : shapes) {
    if (argc > 1 && !strstr(sh.name, argv[1])) continue;
    const int B = 16, M = B * sh.H * sh.H, K = 9 * sh.C;
    const size_t nx = (size_t)M * sh.C;
    float* x = dev_random(nx, 1, 1.0f);
    std::vector<unsigned> words((size_t)B * SFA_AMAX_WORDS, 0u);
    for (int b = 0; b < B; ++b) { const float mx = 0.5f; memcpy(&words[(size_t)b * SFA_AMAX_WORDS], &mx, 4); }
    unsigned *amax_x, *amax_y;
    CK(hipMalloc(&amax_x, words.size() * 4));
    CK(hipMemcpy(amax_x, words.data(), words.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&amax_y, words.size() * 4));
    float* w = dev_random((size_t)sh.N * K, 2, 2.0f / std::sqrt((float)K));
    float* bias = dev_random(sh.N, 3, 0.2f);
    float* res = sh.res ? dev_random((size_t)M * sh.N, 4, 1.0f) : nullptr;
    float* y;
    CK(hipMalloc(&y, (size_t)M * sh.N * 4));
    uint16_t* whp;
    float* winvp;
    split_weights_h3(w, sh.N, K, &whp, &winvp);
    ConvArgs a;
    memset(&a, 0, sizeof a);
    a.nseg = 1;
    make_seg(a.seg[0], x, B, sh.H, sh.H, sh.C, 3, 1, 1);
    a.w = w; a.wh = whp; a.winv = winvp; a.amax_in[0] = amax_x; a.amax_out = amax_y;
    a.bias = bias; a.res = res; a.M = M; a.N = sh.N; a.OH = sh.H; a.OW = sh.H; a.relu = 1; a.Kpad = K; a.y = y;
    a.part = part; a.part_floats = (size_t)16 << 22; a.ksplit = sh.ks;
    const int nblocks = ((M + sh.BM - 1) / sh.BM) * (sh.N / (sh.BM == 128 && sh.N == 64 ? 64 : (sh.N == 512 ? 64 : 128))) * sh.ks;
    const int NW = sh.BM / sh.WM, REC = 2 + 5 * 96 + 2;
    unsigned long long* stp;
    CK(hipMalloc(&stp, (size_t)nblocks * NW * REC * 8 + (1 << 20)));
    CK(hipMemset(stp, 0, (size_t)nblocks * NW * REC * 8));
    a.hout = reinterpret_cast<float*>(stp);
    int rc;
    for (int it = 0; it < 3; ++it) {  // warm (caches, clocks), the last launch's stamps are kept
      if (sh.N == 64) rc = launch_conv_h3s_stamp_cfg<128, 64, 32, EPI_STD, 3, 1166>(a, st);
      else if (sh.N == 512) rc = launch_conv_h3s_stamp_cfg<128, 64, 32, EPI_STD, 3, 1166>(a, st);
      else rc = launch_conv_h3s_stamp_cfg<128, 128, 32, EPI_STD, 3, 1038>(a, st);
      if (rc != SFA_OK) { printf("%s: launch failed\n", sh.name); return 1; }
    }
    CK(hipStreamSynchronize(st));
    std::vector<unsigned long long> h((size_t)nblocks * NW * REC);
    CK(hipMemcpy(h.data(), stp, h.size() * 8, hipMemcpyDeviceToHost));
    const int nks = 3 * 3 * (sh.C / 32) / sh.ks;
    char fn[256];
    snprintf(fn, sizeof fn, "gpurun_out/stamps_%s.bin", sh.name);
    FILE* f = fopen(fn, "wb");
    const int hdr[4] = {nblocks, NW, REC, nks};
    fwrite(hdr, 4, 4, f);
    fwrite(h.data(), 8, h.size(), f);
    fclose(f);
    printf("%s: %d blocks x %d waves, %d k-steps -> %s\n", sh.name, nblocks, NW, nks, fn);
    CK(hipFree(x)); CK(hipFree(amax_x)); CK(hipFree(amax_y)); CK(hipFree(w)); CK(hipFree(bias));
    if (res) CK(hipFree(res));
    CK(hipFree(y)); CK(hipFree(whp)); CK(hipFree(winvp)); CK(hipFree(stp));
  }
  return 0;
}
