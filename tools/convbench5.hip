// Round-5 micro-benchmark of the 3x3/s1 body convs at bs=16, 608x608 (tools only): the product strip
// kernel (conv_h3s_kernel.h) against the persistent strip kernel (conv_h3p_kernel.h), A B A B, every
// candidate's output compared bit for bit with the first one (same products and K order: maxdiff 0),
// with the per-frame output maxima (amax_out) recorded as in the forward.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -pthread tools/convbench5.hip -o tools/convbench5
//   ./tools/convbench5 [iters] [shape substring]
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
#include "experiments/r05/conv_h3p_kernel.h"

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


struct Shape {
  const char* name;
  int B, H, W, C, N;
  bool res;
};
typedef std::function<int(const ConvArgs&, hipStream_t)> Launch;
struct Cand {
  std::string name;
  Launch fn;
};
static float* g_part = nullptr;
static unsigned* g_tick = nullptr;  // split-K tickets (zeroed before every launch, as the forward's memset does)
static const size_t g_part_floats = 64u << 20;
#define CS(BM, BN, WM, OCC, ABL, KS)                                                                  \
  Cand {                                                                                            \
    "h3s " #BM "x" #BN " occ" #OCC " abl" #ABL " ks" #KS, [](const ConvArgs& a, hipStream_t s) {      \
      ConvArgs b = a;                                                                               \
      b.ksplit = KS;                                                                                \
      b.part = g_part;                                                                              \
      b.part_floats = g_part_floats;                                                                \
      return launch_conv_h3s_cfg<BM, BN, WM, EPI_STD, OCC, ABL>(b, s);                              \
    }                                                                                               \
  }
#define CT(BM, BN, WM, OCC, ABL, KS)                                                                  \
  Cand {                                                                                            \
    "h3s " #BM "x" #BN " occ" #OCC " abl" #ABL " ks" #KS " tickets+memset", [](const ConvArgs& a, hipStream_t s) { \
      ConvArgs b = a;                                                                               \
      b.ksplit = KS;                                                                                \
      b.part = g_part;                                                                              \
      b.part_floats = g_part_floats;                                                                \
      b.tile_cnt = g_tick;                                                                          \
      if (hipMemsetAsync(g_tick, 0, 64 * 1024, s) != hipSuccess) return -1;                           \
      return launch_conv_h3s_cfg<BM, BN, WM, EPI_STD, OCC, ABL>(b, s);                              \
    }                                                                                               \
  }
#define CR(BM, BN, WM, OCC, NS, ABL, KS)                                                              \
  Cand {                                                                                            \
    "r3 " #BM "x" #BN " occ" #OCC " st" #NS " abl" #ABL " ks" #KS, [](const ConvArgs& a, hipStream_t s) { \
      ConvArgs b = a;                                                                               \
      b.ksplit = KS;                                                                                \
      b.part = g_part;                                                                              \
      b.part_floats = g_part_floats;                                                                \
      return launch_conv_r3_cfg<BM, BN, WM, EPI_STD, OCC, NS, ABL>(b, s);                           \
    }                                                                                               \
  }
#define CP(BM, BN, WM, OCC, RESPF, KS)                                                                \
  Cand {                                                                                            \
    "h3p " #BM "x" #BN " occ" #OCC " respf" #RESPF " ks" #KS, [](const ConvArgs& a, hipStream_t s) {  \
      ConvArgs b = a;                                                                               \
      b.ksplit = KS;                                                                                \
      b.part = g_part;                                                                              \
      b.part_floats = g_part_floats;                                                                \
      return launch_conv_h3p_cfg<BM, BN, WM, OCC, RESPF>(b, s);                                     \
    }                                                                                               \
  }

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  const char* only = argc > 2 ? argv[2] : nullptr;
  std::vector<Shape> shapes = {
      {"layer1 3x3 64->64 +res", 16, 152, 152, 64, 64, true},
      {"layer2 3x3 128->128", 16, 76, 76, 128, 128, false},
      {"layer2 3x3 128->128 +res", 16, 76, 76, 128, 128, true},
      {"layer3 3x3 256->256", 16, 38, 38, 256, 256, false},
      {"layer3 3x3 256->256 +res", 16, 38, 38, 256, 256, true},
      {"layer4 3x3 512->512", 16, 19, 19, 512, 512, false},
  };
  // round 5: 64 x 64 tiles at 4 blocks / CU (4 waves per SIMD) against the product 128 x 64 at 3
  // (late round 5: 256-row tiles, 8 waves, 1 / 2 blocks per CU: the W tile amortised over twice the rows)
  std::vector<Cand> l1 = {CS(128, 64, 32, 3, 142, 1), CS(256, 64, 32, 1, 142, 1), CS(256, 64, 32, 2, 142, 1),
                          CS(128, 64, 32, 3, 142, 1), CS(256, 64, 32, 1, 142, 1), CS(256, 64, 32, 2, 142, 1)};
  // round 5: the pre-split strip (4) and the residual prefetch (128) on the 128-wide tiles
  std::vector<Cand> l2 = {CS(128, 128, 32, 2, 10, 1), CS(128, 128, 32, 2, 14, 1), CS(128, 128, 32, 2, 142, 1),
                          CS(128, 128, 32, 2, 10, 1), CS(128, 128, 32, 2, 14, 1), CS(128, 128, 32, 2, 142, 1)};
  // round 5: the heads' register-A kernel (half-tile stagger, 3-stage W ring) on 256-wide tiles, the
  // grid filled by split-K (reduce launch)
  std::vector<Cand> l3 = {CS(64, 128, 16, 3, 10, 1), CS(64, 128, 16, 3, 14, 1), CS(64, 128, 16, 3, 142, 1),
                          CS(64, 128, 16, 3, 10, 1), CS(64, 128, 16, 3, 14, 1), CS(64, 128, 16, 3, 142, 1)};
  std::vector<Cand> l4 = {CS(128, 64, 32, 3, 142, 2), CT(128, 64, 32, 3, 142, 2), CR(192, 256, 32, 1, 3, 1603844, 4),
                          CR(256, 256, 32, 1, 3, 1603844, 6), CR(192, 256, 32, 1, 3, 1603844, 3),
                          CS(128, 64, 32, 3, 142, 2), CT(128, 64, 32, 3, 142, 2), CR(192, 256, 32, 1, 3, 1603844, 4)};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  CK(hipMalloc(&g_part, g_part_floats * 4));
  CK(hipMalloc(&g_tick, 64 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  unsigned* amax_y;
  CK(hipMalloc(&amax_y, (size_t)64 * SFA_AMAX_WORDS * 4));
  for (const Shape& sh : shapes) {
    if (only && !strstr(sh.name, only)) continue;
    const int OH = sh.H, OW = sh.W, M = sh.B * OH * OW, K = 9 * sh.C, Kpad = K;
    const size_t nx = (size_t)sh.B * sh.H * sh.W * sh.C;
    float* x = dev_random(nx, 1, 1.0f);
    unsigned* amax_x;
    {
      std::vector<float> hx(nx);
      CK(hipMemcpy(hx.data(), x, nx * 4, hipMemcpyDeviceToHost));
      std::vector<unsigned> words((size_t)sh.B * SFA_AMAX_WORDS, 0u);
      const size_t per = nx / sh.B;
      for (int b = 0; b < sh.B; ++b) {
        float mx = 0.f;
        for (size_t i = 0; i < per; ++i) mx = std::max(mx, std::fabs(hx[b * per + i]));
        memcpy(&words[(size_t)b * SFA_AMAX_WORDS + SFA_AMAX_STRIDE * 3], &mx, 4);
      }
      CK(hipMalloc(&amax_x, words.size() * 4));
      CK(hipMemcpy(amax_x, words.data(), words.size() * 4, hipMemcpyHostToDevice));
    }
    float* w = dev_random((size_t)sh.N * Kpad, 2, 2.0f / std::sqrt((float)K));
    float* b = dev_random(sh.N, 3, 0.2f);
    float* res = sh.res ? dev_random((size_t)M * sh.N, 4, 1.0f) : nullptr;
    const size_t ysz = (size_t)M * sh.N;
    float* y;
    CK(hipMalloc(&y, ysz * 4));
    uint16_t* whp = nullptr;
    float* winvp = nullptr;
    split_weights_h3(w, sh.N, Kpad, &whp, &winvp);
    ConvArgs a;
    memset(&a, 0, sizeof a);
    a.nseg = 1;
    make_seg(a.seg[0], x, sh.B, sh.H, sh.W, sh.C, 3, 1, 1);
    a.w = w;
    a.wh = whp;
    a.winv = winvp;
    a.amax_in[0] = amax_x;
    a.amax_out = amax_y;
    a.bias = b;
    a.res = res;
    a.M = M;
    a.N = sh.N;
    a.OH = OH;
    a.OW = OW;
    a.relu = 1;
    a.Kpad = Kpad;
    a.y = y;
    const double flop = 2.0 * M * sh.N * (double)K;
    std::vector<Cand>& cands = sh.C == 64 ? l1 : sh.C == 128 ? l2 : sh.C == 256 ? l3 : l4;
    printf("\n== %s  M=%d N=%d K=%d  (%.2f GFLOP)\n", sh.name, M, sh.N, K, flop / 1e9);
    std::vector<float> ref, got;
    std::vector<unsigned> aref, agot;
    for (Cand& c : cands) {
      CK(hipMemset(y, 0, ysz * 4));
      CK(hipMemset(amax_y, 0, (size_t)64 * SFA_AMAX_WORDS * 4));
      if (c.fn(a, st) != SFA_OK) {
        printf("  %-36s unsupported\n", c.name.c_str());
        continue;
      }
      CK(hipStreamSynchronize(st));
      got.resize(ysz);
      CK(hipMemcpy(got.data(), y, ysz * 4, hipMemcpyDeviceToHost));
      agot.resize((size_t)sh.B * SFA_AMAX_WORDS);
      CK(hipMemcpy(agot.data(), amax_y, agot.size() * 4, hipMemcpyDeviceToHost));
      std::vector<unsigned> fr(sh.B, 0u);  // per-frame max over the shards
      for (int f = 0; f < sh.B; ++f)
        for (int j = 0; j < SFA_AMAX_SHARDS; ++j) fr[f] = std::max(fr[f], agot[(size_t)f * SFA_AMAX_WORDS + j * SFA_AMAX_STRIDE]);
      double maxd = 0;
      size_t ndiff = 0;
      bool amax_ok = true;
      if (ref.empty()) {
        ref = got;
        aref = fr;
      } else {
        for (size_t i = 0; i < ysz; ++i) {
          if (memcmp(&got[i], &ref[i], 4)) ++ndiff;
          maxd = std::max(maxd, (double)std::fabs(got[i] - ref[i]));
        }
        amax_ok = fr == aref;
      }
      std::vector<float> ms;
      for (int it = 0; it < iters; ++it) {
        CK(hipEventRecord(e0, st));
        c.fn(a, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
      }
      std::sort(ms.begin(), ms.end());
      const float med = ms[ms.size() / 2];
      printf("  %-36s %9.1f us  %7.1f TF/s  bits-differ %zu  maxdiff %.2e  amax %s\n", c.name.c_str(), med * 1e3,
             flop / (med * 1e-3) / 1e12, ndiff, maxd, amax_ok ? "equal" : "DIFFER");
    }
    CK(hipFree(x));
    CK(hipFree(amax_x));
    CK(hipFree(w));
    CK(hipFree(b));
    if (res) CK(hipFree(res));
    CK(hipFree(y));
    CK(hipFree(whp));
    CK(hipFree(winvp));
  }
  return 0;
}
