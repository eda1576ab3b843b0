// Round-4 micro-benchmark of the PRODUCT conv kernels (csrc headers) and their round-4 variants on
// the KFPN layer shapes at bs=16, 608x608 (tools only; tools/convbench.hip keeps the round-3 variants).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -pthread -I<pkg>/csrc tools/convbench4.hip -o tools/convbench4
//   ./tools/convbench [iters] [shape substring]; env SUSTAIN=<s>: also back-to-back for s seconds
//   per candidate with the board's clock and power read mid-run (rocm-smi)
//   ./tools/convbench [iters]
// Every candidate's output is compared with the first candidate's (same math,
// different tiling -> differences only from summation order).
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
#include "experiments/r04/conv_wres_kernel.h"
#include "experiments/r04/stem_band_kernel.h"
#include "experiments/r04/conv_ws_kernel.h"

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
  int B, H, W, C, k, stride, pad, N;
  bool head, res;
};

typedef std::function<int(const ConvArgs&, hipStream_t)> Launch;
struct Cand {
  std::string name;
  int BK;
  Launch fn;
};
static float* g_part = nullptr;
static const size_t g_part_floats = 64u << 20;
#define CANDTK(BM, BN, WM, EPI, OCC, ABL, KS)                                                      \
  Cand {                                                                                          \
    "h3strip " #BM "x" #BN " w" #WM " occ" #OCC " abl" #ABL " ks" #KS, 32,                          \
        [](const ConvArgs& a, hipStream_t s) {                                                    \
          ConvArgs b = a;                                                                         \
          b.ksplit = KS;                                                                          \
          b.part = g_part;                                                                        \
          b.part_floats = g_part_floats;                                                          \
          return launch_conv_h3s_cfg<BM, BN, WM, EPI, OCC, ABL>(b, s);                            \
        }                                                                                         \
  }
#define CANDH3(BM, BN, WM, OCC, NK, NST, KS)                                                        \
  Cand {                                                                                          \
    "h3 " #BM "x" #BN " w" #WM " occ" #OCC " st" #NST " ks" #KS, 32, [](const ConvArgs& a, hipStream_t s) {   \
      ConvArgs b = a;                                                                             \
      b.ksplit = KS;                                                                              \
      b.part = g_part;                                                                            \
      b.part_floats = g_part_floats;                                                              \
      return launch_conv_h3_cfg<BM, BN, WM, EPI_STD, OCC, NK, NST, false, 2, 1>(b, s);             \
    }                                                                                             \
  }
// the fp16x3 stems (NCHW3 input planes, pooled output): band kernel / round-3 patch kernel + merge
#define CANDSTEM(FORM)                                                                            \
  Cand {                                                                                          \
    FORM == 2 ? "h3 stem band" : "h3 stem patch+merge", 32, [](const ConvArgs& a, hipStream_t s) { \
      ConvArgs b = a;                                                                             \
      b.stem_in = STEM_IN_NCHW3;                                                                  \
      b.part = g_part;                                                                            \
      b.part_floats = g_part_floats;                                                              \
      return FORM == 2 ? launch_stem_band(b, s) : launch_stem_patch_pool(b, s);                  \
    }                                                                                             \
  }
#define CANDR(BM, BN, WM, EPI, OCC, NS, ABL, KS)                                                    \
  Cand {                                                                                          \
    "h3r " #BM "x" #BN " w" #WM " occ" #OCC " st" #NS " abl" #ABL " ks" #KS, 32,                    \
        [](const ConvArgs& a, hipStream_t s) {                                                    \
          ConvArgs b = a;                                                                         \
          b.ksplit = KS;                                                                          \
          b.part = g_part;                                                                        \
          b.part_floats = g_part_floats;                                                          \
          return launch_conv_r3_cfg<BM, BN, WM, EPI, OCC, NS, ABL>(b, s);                         \
        }                                                                                         \
  }

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  const char* only = argc > 2 ? argv[2] : nullptr;
  const double sustain = getenv("SUSTAIN") ? atof(getenv("SUSTAIN")) : 0.0;
  std::vector<Shape> shapes = {
      {"stem 7x7/2 4->64", 16, 608, 608, 4, 7, 2, 3, 64, false, false},
      {"layer1 3x3 64->64 +res", 16, 152, 152, 64, 3, 1, 1, 64, false, true},
      {"layer2 3x3 128->128", 16, 76, 76, 128, 3, 1, 1, 128, false, false},
      {"layer3 3x3 256->256", 16, 38, 38, 256, 3, 1, 1, 256, false, false},
      {"layer4 3x3 512->512", 16, 19, 19, 512, 3, 1, 1, 512, false, false},
      {"s2 layer2.0.conv1 3x3/2 64->128", 16, 152, 152, 64, 3, 2, 1, 128, false, false},
      {"s2 layer3.0.conv1 3x3/2 128->256", 16, 76, 76, 128, 3, 2, 1, 256, false, false},
      {"s2 layer4.0.conv1 3x3/2 256->512", 16, 38, 38, 256, 3, 2, 1, 512, false, false},
      {"head L1 3x3 128->5x64", 16, 152, 152, 128, 3, 1, 1, 320, true, false},
      {"head L2 3x3 64->5x64", 16, 152, 152, 64, 3, 1, 1, 320, true, false},
      {"head L0 3x3 256->5x64", 16, 76, 76, 256, 3, 1, 1, 320, true, false},
      {"head tiny 3x3 8->5x64 (epilogue cost)", 16, 152, 152, 8, 3, 1, 1, 320, true, false},
  };
  // round 4: register-staged W (ABL 256) against the product strip kernels, A B A B
  std::vector<Cand> n64 = {
      CANDTK(128, 64, 32, EPI_STD, 3, 142, 1), CANDTK(128, 64, 32, EPI_STD, 3, 398, 1),
      CANDTK(128, 64, 32, EPI_STD, 3, 142, 1), CANDTK(128, 64, 32, EPI_STD, 3, 398, 1),
  };
  n64.push_back(Cand{"h3 weight-stationary rows", 32, [](const ConvArgs& a, hipStream_t s) { return launch_conv_ws(a, s); }});
  n64.push_back(Cand{"h3 weight-stationary rows", 32, [](const ConvArgs& a, hipStream_t s) { return launch_conv_ws(a, s); }});
  // round 4 (late): whole weight image resident in LDS, barrier-free register-A waves
  n64.clear();
  n64.push_back(CANDTK(128, 64, 32, EPI_STD, 3, 142, 1));
  n64.push_back(Cand{"h3 wres nw8 pd2", 32, [](const ConvArgs& a, hipStream_t s) { return launch_conv_wres_cfg<64, 8, 2>(a, s); }});
  n64.push_back(Cand{"h3 wres nw8 pd1", 32, [](const ConvArgs& a, hipStream_t s) { return launch_conv_wres_cfg<64, 8, 1>(a, s); }});
  n64.push_back(Cand{"h3 wres nw12 pd2", 32, [](const ConvArgs& a, hipStream_t s) { return launch_conv_wres_cfg<64, 12, 2>(a, s); }});
  n64.push_back(CANDTK(128, 64, 32, EPI_STD, 3, 142, 1));
  n64.push_back(Cand{"h3 wres nw8 pd2", 32, [](const ConvArgs& a, hipStream_t s) { return launch_conv_wres_cfg<64, 8, 2>(a, s); }});
  std::vector<Cand> stem = {CANDSTEM(1), CANDSTEM(2), CANDSTEM(1), CANDSTEM(2)};
  std::vector<Cand> nbig = {
      CANDTK(128, 128, 32, EPI_STD, 2, 10, 1), CANDTK(128, 128, 32, EPI_STD, 2, 266, 1),
      CANDTK(128, 128, 32, EPI_STD, 2, 10, 1), CANDTK(128, 128, 32, EPI_STD, 2, 266, 1),
      CANDTK(64, 128, 16, EPI_STD, 3, 10, 1), CANDTK(128, 64, 32, EPI_STD, 3, 10, 1),
      // round 4 (late): split-K grids (layer2: 722 128 x 128 tiles = 1.41 rounds of 512 slots)
      CANDTK(128, 128, 32, EPI_STD, 2, 10, 2), CANDTK(64, 128, 16, EPI_STD, 3, 10, 2),
      CANDTK(128, 64, 32, EPI_STD, 3, 142, 2), CANDTK(128, 128, 32, EPI_STD, 2, 10, 4),
      CANDTK(128, 128, 32, EPI_STD, 2, 10, 1),
      // round 4 (late): the heads' register-A form with the half-tile stagger and the 3-stage W ring
      // (R3_HEAD_STAG without the packed head epilogue) on the 3x3/s1 body convs
      CANDR(128, 128, 32, EPI_STD, 2, 3, 1603844, 1), CANDR(256, 128, 32, EPI_STD, 1, 3, 1603844, 1),
      CANDR(256, 128, 32, EPI_STD, 2, 3, 1603844, 1), CANDR(128, 128, 32, EPI_STD, 2, 2, 526592, 1),
      CANDTK(128, 128, 32, EPI_STD, 2, 10, 1),
  };
  std::vector<Cand> n512 = {
      CANDTK(128, 128, 32, EPI_STD, 2, 10, 2), CANDTK(128, 128, 32, EPI_STD, 2, 266, 2),
      CANDTK(128, 128, 32, EPI_STD, 2, 10, 2), CANDTK(128, 128, 32, EPI_STD, 2, 266, 2),
      // round 4: grids that fill the chip without split-K (no reduce launch)
      CANDTK(64, 128, 16, EPI_STD, 3, 10, 1), CANDTK(128, 64, 32, EPI_STD, 3, 10, 1),
      CANDTK(128, 64, 32, EPI_STD, 3, 142, 1),
      // round 4 (late): the split-K grids of the other tile shapes (3 blocks / CU) and deeper splits
      CANDTK(64, 128, 16, EPI_STD, 3, 10, 2), CANDTK(128, 64, 32, EPI_STD, 3, 10, 2),
      CANDTK(128, 64, 32, EPI_STD, 3, 142, 2), CANDTK(128, 128, 32, EPI_STD, 2, 10, 3),
      CANDTK(128, 128, 32, EPI_STD, 2, 10, 4), CANDTK(64, 128, 16, EPI_STD, 3, 10, 3),
      CANDTK(64, 128, 16, EPI_STD, 3, 10, 4), CANDTK(128, 128, 32, EPI_STD, 2, 10, 2),
  };
  // stride-2 conv1 of layers 2/3 (and 4): the product picks conv_r3 128 x 128 for the big-M layer2 and
  // conv_h3 128 x 128 for the others (conv.hip); both, and 64-row conv_r3 tiles, on each shape
  std::vector<Cand> s2 = {
      CANDR(128, 128, 32, EPI_STD, 2, 2, 526592, 1), CANDH3(128, 128, 32, 2, 32, 2, 1),
      CANDR(64, 128, 16, EPI_STD, 3, 2, 526592, 1), CANDR(64, 128, 32, EPI_STD, 4, 2, 526592, 1),
      CANDR(128, 128, 32, EPI_STD, 2, 2, 526592, 1), CANDH3(128, 128, 32, 2, 32, 2, 1),
      // round 5: deeper W / A rings for conv_h3 (one block per CU)
      CANDH3(128, 128, 32, 1, 32, 3, 1), CANDH3(128, 128, 32, 1, 32, 4, 1), CANDH3(128, 128, 32, 2, 32, 2, 1),
      // round 5: split-K 2 / 3 for the stride-2 convs (362 / 722 tiles for 512 / 768 slots without)
      CANDH3(128, 128, 32, 2, 32, 2, 2), CANDH3(128, 128, 32, 2, 32, 2, 3),
      CANDR(64, 128, 16, EPI_STD, 3, 2, 526592, 2), CANDR(128, 128, 32, EPI_STD, 2, 2, 526592, 2),
  };
  // layer4.0.conv1 (M 5776, N 512): the product's conv_h3 128 x 128 with split-K 2 against other
  // splits and the 64-row conv_r3 tiles with split-K
  std::vector<Cand> s2n512 = {
      CANDH3(128, 128, 32, 2, 32, 2, 2), CANDR(64, 128, 16, EPI_STD, 3, 2, 526592, 2),
      CANDR(128, 128, 32, EPI_STD, 2, 2, 526592, 2), CANDH3(128, 128, 32, 2, 32, 2, 3),
      CANDH3(128, 128, 32, 2, 32, 2, 4), CANDR(64, 128, 16, EPI_STD, 3, 2, 526592, 3),
      CANDR(64, 128, 16, EPI_STD, 3, 2, 526592, 4), CANDH3(128, 128, 32, 2, 32, 2, 2),
      CANDH3(128, 128, 32, 1, 32, 3, 2), CANDH3(128, 128, 32, 1, 32, 4, 2), CANDH3(128, 128, 32, 2, 32, 2, 2),
  };
  std::vector<Cand> heads = {
      CANDR(256, 320, 32, EPI_HEAD, 1, 3, 1669380, 1),
  };
  hipStream_t st;
  CK(hipStreamCreate(&st));
  CK(hipMalloc(&g_part, g_part_floats * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& sh : shapes) {
    if (only && !strstr(sh.name, only)) continue;
    const int OH = (sh.H + 2 * sh.pad - sh.k) / sh.stride + 1;
    const int OW = (sh.W + 2 * sh.pad - sh.k) / sh.stride + 1;
    const int M = sh.B * OH * OW;
    const int K = sh.k * sh.k * sh.C;
    const int Kpad = (K + 31) / 32 * 32;
    const size_t nx = (size_t)sh.B * sh.H * sh.W * sh.C;
    float* x = dev_random(nx, 1, 1.0f);
    unsigned* amax_x;  // per-frame max |x| (conv.h fp16x3 layout)
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
    float* hw1 = dev_random(8 * 4 * 64, 5, 0.25f);
    float* hb1 = dev_random(8 * 4, 6, 0.2f);
    const int nh = sh.N / 64;
    const size_t ysz = sh.head ? (size_t)11 * M : (size_t)M * sh.N;
    float *y, *y0;
    CK(hipMalloc(&y, ysz * 4));
    CK(hipMalloc(&y0, ysz * 4));
    // zero weight columns beyond K so Kpad=224/208 variants agree
    {
      std::vector<float> hwv((size_t)sh.N * Kpad);
      CK(hipMemcpy(hwv.data(), w, hwv.size() * 4, hipMemcpyDeviceToHost));
      for (int n = 0; n < sh.N; ++n)
        for (int k = K; k < Kpad; ++k) hwv[(size_t)n * Kpad + k] = 0.f;
      CK(hipMemcpy(w, hwv.data(), hwv.size() * 4, hipMemcpyHostToDevice));
    }
    ConvArgs a;
    memset(&a, 0, sizeof a);
    a.nseg = 1;
    make_seg(a.seg[0], x, sh.B, sh.H, sh.W, sh.C, sh.k, sh.stride, sh.pad);
    a.w = w;
    a.bias = b;
    a.res = res;
    a.M = M;
    a.N = sh.N;
    a.OH = OH;
    a.OW = OW;
    a.relu = 1;
    a.hw1 = hw1;
    a.hb1 = hb1;
    int off = 0;
    const int hc[5] = {3, 2, 2, 1, 3};
    for (int j = 0; j < nh; ++j) {
      a.hch[j] = hc[j % 5];
      a.hoff[j] = off;
      off += a.hch[j];
    }
    const double flop = 2.0 * M * sh.N * (double)K;
    std::vector<Cand>& cands = sh.head ? heads : sh.C == 4 ? stem : sh.stride == 2 ? (sh.N == 512 ? s2n512 : s2) : (sh.N == 64 ? n64 : sh.N == 512 ? n512 : nbig);
    printf("\n== %s  M=%d N=%d K=%d  (%.2f GFLOP)\n", sh.name, M, sh.N, K, flop / 1e9);
    std::vector<float> ref, got;
    ref.clear();
    for (size_t ci = 0; ci < cands.size(); ++ci) {
      Cand& c = cands[ci];
      a.Kpad = c.BK == 16 ? (K + 15) / 16 * 16 : Kpad;
      // weights are [N][Kpad]; re-stride when Kpad differs from the allocation
      float* wv = w;
      if (a.Kpad != Kpad) {
        std::vector<float> hwv((size_t)sh.N * Kpad), hw2((size_t)sh.N * a.Kpad);
        CK(hipMemcpy(hwv.data(), w, hwv.size() * 4, hipMemcpyDeviceToHost));
        for (int n = 0; n < sh.N; ++n)
          for (int k = 0; k < a.Kpad; ++k) hw2[(size_t)n * a.Kpad + k] = hwv[(size_t)n * Kpad + k];
        CK(hipMalloc(&wv, hw2.size() * 4));
        CK(hipMemcpy(wv, hw2.data(), hw2.size() * 4, hipMemcpyHostToDevice));
      }
      a.w = wv;
      a.wx = c.name.rfind("x6", 0) == 0 ? split_weights(wv, (size_t)sh.N * a.Kpad) : nullptr;
      uint16_t* whp = nullptr;
      float* winvp = nullptr;
      if (c.name.rfind("h3", 0) == 0) split_weights_h3(wv, sh.N, a.Kpad, &whp, &winvp);
      a.wh = whp;
      a.winv = winvp;
      a.amax_in[0] = whp ? amax_x : nullptr;
      a.y = y;
      a.hout = y;
      CK(hipMemset(y, 0, ysz * 4));
      if (c.fn(a, st) != SFA_OK) {
        printf("  %-32s unsupported\n", c.name.c_str());
        continue;
      }
      CK(hipStreamSynchronize(st));
      got.resize(ysz);
      CK(hipMemcpy(got.data(), y, ysz * 4, hipMemcpyDeviceToHost));
      double maxd = 0, maxr = 0;
      if (ref.empty()) {  // the first supported candidate is the reference
        ref = got;
      } else {
        for (size_t i = 0; i < ysz; ++i) {
          maxd = std::max(maxd, (double)std::fabs(got[i] - ref[i]));
          maxr = std::max(maxr, (double)std::fabs(ref[i]));
        }
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
      printf("  %-32s %9.1f us  %7.1f TF/s  maxdiff %.2e (|ref| %.2e)\n", c.name.c_str(), med * 1e3,
             flop / (med * 1e-3) / 1e12, maxd, maxr);
      if (sustain > 0) {  // back-to-back launches for `sustain` s (board at its power limit)
        std::string smi;
        std::thread probe([&] {
          std::this_thread::sleep_for(std::chrono::milliseconds((int)(sustain * 600)));
          FILE* f = popen("rocm-smi --showpower --showclocks 2>/dev/null | grep -E 'sclk|Power \\(W\\)'", "r");
          if (!f) return;
          char buf[256];
          while (fgets(buf, sizeof buf, f)) {
            std::string l(buf);
            const size_t k = l.find_last_of(':');
            smi += (k == std::string::npos ? l : l.substr(k + 1));
          }
          pclose(f);
          for (char& ch : smi)
            if (ch == '\n' || ch == '\t') ch = ' ';
        });
        int n = 0;
        float tot = 0;
        CK(hipEventRecord(e0, st));
        while (tot < sustain * 1000) {
          for (int k = 0; k < 20; ++k) c.fn(a, st);
          n += 20;
          CK(hipEventRecord(e1, st));
          CK(hipEventSynchronize(e1));
          CK(hipEventElapsedTime(&tot, e0, e1));
        }
        probe.join();
        const double per = tot / n;
        printf("  %-32s sustained %.1f us  %7.1f TF/s  [smi:%s]\n", "", per * 1e3, flop / (per * 1e-3) / 1e12,
               smi.c_str());
      }
      if (wv != w) CK(hipFree(wv));
      if (a.wx) CK(hipFree(const_cast<uint16_t*>(a.wx)));
      if (whp) CK(hipFree(whp));
      if (winvp) CK(hipFree(winvp));
    }
    CK(hipFree(x));
    CK(hipFree(amax_x));
    CK(hipFree(w));
    CK(hipFree(b));
    if (res) CK(hipFree(res));
    CK(hipFree(hw1));
    CK(hipFree(hb1));
    CK(hipFree(y));
    CK(hipFree(y0));
  }
  return 0;
}
