// Power-capped MFMA throughput: v_mfma_f32_16x16x32_f16 vs v_mfma_f32_32x32x16_f16 chains on
// random operands over the whole chip (2 waves per SIMD), sustained for a few seconds each, to
// see which shape delivers more FLOP per joule once the board sits at its power limit.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/mfma_power.hip -o tools/micro/mfma_power
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int SHAPE, int NV = 0>  // 0: 16x16x32, 1: 32x32x16; NV: f32 FMAs (VALU) per MFMA (SHAPE 0)
__global__ void __launch_bounds__(512, 1) mfma_loop(const h8* __restrict__ in, float* __restrict__ out, int iters) {
  const int lane = threadIdx.x & 63;
  float vq[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) vq[i] = (float)in[lane * 8 + i][0];
  const float vm = (float)in[lane][1], va = (float)in[lane][2];
  h8 a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = in[(blockIdx.x * 8 + i) * 64 + lane];
    b[i] = in[(blockIdx.x * 8 + 4 + i) * 64 + lane];
  }
  if constexpr (SHAPE == 0) {
    f4 c[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) c[i] = f4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 16; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i & 3], b[i >> 2], c[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        c[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(i + 1) & 3], b[i >> 2], c[i], 0, 0, 0);
        if constexpr (NV > 0) {
#pragma unroll
          for (int v = 0; v < NV; ++v)  // one VALU instruction each (no packing)
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(vq[(i * NV + v) & 7]) : "v"(vm), "v"(va));
        }
      }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += vq[i];
#pragma unroll
    for (int i = 0; i < 16; ++i) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
    out[blockIdx.x * 512 + threadIdx.x] = s;
  } else {
    f16v c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) c[i][j] = 0;
    for (int it = 0; it < iters; ++it) {
      // same FLOPs per iteration as SHAPE 0: 32 x 16x16x32 = 16 x 32x32x16
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[(i + r) & 3], b[r], c[i], 0, 0, 0);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) s += c[i][j];
    out[blockIdx.x * 512 + threadIdx.x] = s;
  }
}

int main(int argc, char** argv) {
  const double secs = argc > 1 ? atof(argv[1]) : 4.0;
  const int blocks = 256, iters = 4000;
  std::vector<_Float16> h((size_t)blocks * 8 * 64 * 8);
  srand(1);
  for (auto& v : h) v = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 2.0f);
  h8* in;
  float* out;
  CK(hipMalloc(&in, h.size() * 2));
  CK(hipMalloc(&out, (size_t)blocks * 512 * 4));
  CK(hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double flop = (double)blocks * 8 * iters * 32 * 16384;  // per launch
  const char* names[5] = {"16x16x32", "32x32x16", "16x16x32 +0.5 VALU/MFMA", "16x16x32 +1 VALU/MFMA",
                          "16x16x32 +2 VALU/MFMA"};
  for (int shape = 0; shape < 5; ++shape) {
    for (int rep = 0; rep < 1 + (shape < 2); ++rep) {
      int launches = 0;
      float total_ms = 0;
      CK(hipEventRecord(e0));
      while (total_ms < secs * 1000) {
        for (int k = 0; k < 20; ++k) {
          if (shape == 0) mfma_loop<0><<<blocks, 512>>>(in, out, iters);
          else if (shape == 1) mfma_loop<1><<<blocks, 512>>>(in, out, iters);
          else if (shape == 2) mfma_loop<0, 1><<<blocks, 512>>>(in, out, iters);
          else if (shape == 3) mfma_loop<0, 2><<<blocks, 512>>>(in, out, iters);
          else mfma_loop<0, 4><<<blocks, 512>>>(in, out, iters);
        }
        launches += 20;
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&total_ms, e0, e1));
      }
      printf("%s rep %d: %.1f TFLOP/s dense fp16 over %.2f s (%d launches)\n", names[shape], rep, flop * launches / (total_ms * 1e-3) / 1e12, total_ms * 1e-3,
             launches);
      fflush(stdout);
    }
  }
  return 0;
}
