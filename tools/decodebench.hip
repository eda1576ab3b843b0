// Decode micro-benchmark (timing + ablations of the band-parallel decode kernels).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/decodebench.hip -o tools/decodebench
//   ./tools/decodebench [reps]
// B = 16, C = 3, 152 x 152, K = 50, random logits (apply_sigmoid = 1): the bench's decode.
#include "../lidar-image_object-detection_-fpn_resnet-yolov8_amd/csrc/decode.hip"

#include <cstdlib>
#include <vector>

namespace sfa {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fprintf(stderr, "\n");
}
}  // namespace sfa

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  const int B = 16, C = 3, H = 152, W = 152, K = 50;
  const size_t hw = (size_t)H * W;
  std::vector<float> h((size_t)B * 11 * hw);
  unsigned x = 12345;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = ((x >> 8) / 16777216.0f) * 12.f - 8.f;
  }
  float* d;
  CK(hipMalloc(&d, h.size() * 4));
  CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const float* hm = d;
  const float* off = d + (size_t)B * 3 * hw;
  const float* dr = d + (size_t)B * 5 * hw;
  const float* zz = d + (size_t)B * 7 * hw;
  const float* dm = d + (size_t)B * 8 * hw;
  float* dets;
  CK(hipMalloc(&dets, (size_t)B * K * 10 * 4));
  size_t wsb = sfa_decode_workspace_size(B, C, K);
  void* ws;
  CK(hipMalloc(&ws, wsb));
  int S, R;
  band_plan(C, H, W, K, &S, &R);
  const size_t nb = (size_t)B * C * S * K;
  auto* bk = reinterpret_cast<unsigned*>(ws);
  auto* bi = reinterpret_cast<int*>(reinterpret_cast<char*>(ws) + align_up(nb * sizeof(unsigned), 256));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto fn) {
    for (int i = 0; i < 10; ++i) fn();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) fn();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-44s %8.2f us\n", name, 1e3f * ms / reps);
  };
  printf("S = %d bands of R = %d rows\n", S, R);
  time("sfa_decode (band topk + merge)", [&] {
    sfa_decode(hm, off, dr, zz, dm, B, C, H, W, K, 1, dets, ws, wsb, nullptr);
  });
#define BAND(ABL)                                                                                       \
  time("band_topk<" #ABL ">", [&] {                                                                     \
    hipLaunchKernelGGL(decode_band_topk_kernel<ABL>, dim3(S, C, B), dim3(kBandThreads), 0, 0, hm, C, H, W, K, R, 1, bk, bi); \
  })
  BAND(0);
  BAND(1);
  BAND(2);
  BAND(4);
  BAND(8);
  BAND(15);
  // valid band lists for the merge (the ablations above leave garbage behind)
  hipLaunchKernelGGL(decode_band_topk_kernel<0>, dim3(S, C, B), dim3(kBandThreads), 0, 0, hm, C, H, W, K, R, 1, bk, bi);
  CK(hipDeviceSynchronize());
  time("band_merge_gather", [&] {
    hipLaunchKernelGGL(decode_band_merge_gather_kernel, dim3(B), dim3(1024), 0, 0, bk, bi, C, S, K, H, W, 1, off, dr,
                       zz, dm, dets);
  });
  CK(hipDeviceSynchronize());
  time("old: class_topk (1 block per class)", [&] {
    hipLaunchKernelGGL(decode_class_topk_kernel<true>, dim3(B * C), dim3(kDecThreads), 0, 0, hm, C, H, W, K, 1, bk, bi);
  });
  time("old: merge_gather", [&] {
    hipLaunchKernelGGL(decode_merge_gather_kernel, dim3(B), dim3(256), 0, 0, bk, bi, C, K, H, W, 1, off, dr, zz, dm,
                       dets);
  });
  return 0;
}
