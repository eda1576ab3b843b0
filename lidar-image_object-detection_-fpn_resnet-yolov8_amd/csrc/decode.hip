// CenterNet decode: utils/evaluation_utils.py:77-105 (_nms :21-26, _topk :47-62,
// _transpose_and_gather_feat :40-44), with utils/torch_utils.py:44-45 _sigmoid
// optionally fused on the fly.
//
// Kernel 1 — one 1024-thread workgroup per (frame, class):
//   the class map is staged whole in LDS (152x152 f32 = 90 KiB), sigmoid+clamp
//   applied if asked, 3x3 peak test against the LDS neighbourhood (-inf padding,
//   plateaus survive: keep = (max == v)), then a block radix-select over the
//   order-preserving u32 key of each peak value (4 MSB-first 8-bit passes with
//   an LDS histogram) finds the K-th largest value T; all keys > T plus the
//   lowest-index keys == T (block prefix scan over contiguous index ranges) are
//   the class's top K, ranked by (value desc, index asc).
// Kernel 2 — one workgroup per frame: the C*K survivors are ranked by
//   (value desc, class*K + rank asc) — torch's second topk — and the K winners
//   gather offset / direction / z / dim at their pixel into (K, 10) rows.
// Integer selection is exact; outputs are bit-exact given identical maps.
#include "common.h"

namespace sfa {

constexpr int kDecThreads = 1024;
constexpr int kDecMaxHW = 36864;  // 144 KiB of LDS
constexpr int kDecMaxK = 256;

__device__ __forceinline__ float sigmoid_clamp_f(float x) {
  const float s = 1.0f / (1.0f + expf(-x));
  return fminf(fmaxf(s, 1e-4f), 1.0f - 1e-4f);
}

// Order-preserving map float -> u32 (larger float -> larger key); -0 == +0.
__device__ __forceinline__ unsigned fkey(float v) {
  unsigned u = __float_as_uint(v == 0.f ? 0.f : v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Block-wide exclusive scan of one int per thread (1024 threads = 16 waves).
__device__ int block_excl_scan(int v, int* wsum /*[16]*/, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  if (wave == 0) {
    int s = lane < 16 ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int y = __shfl_up(s, o, 64);
      if (lane >= o) s += y;
    }
    if (lane < 16) wsum[lane] = s;  // inclusive
  }
  __syncthreads();
  const int before = wave ? wsum[wave - 1] : 0;
  if (total) *total = wsum[15];
  return before + x - v;
}

__global__ void __launch_bounds__(kDecThreads) decode_class_topk_kernel(
    const float* __restrict__ hm, int C, int H, int W, int K, int apply_sigmoid,
    unsigned* __restrict__ cand_key, int* __restrict__ cand_idx) {
  __shared__ __attribute__((aligned(16))) float heat[kDecMaxHW];  // class map, then peak map
  __shared__ unsigned hist[256];
  __shared__ int wsum[16];
  __shared__ int misc[8];
  __shared__ unsigned sel_key[kDecMaxK];
  __shared__ int sel_idx[kDecMaxK];
  const int HW = H * W;

  const int bc = blockIdx.x;  // frame * C + class
  const float* src = hm + (size_t)bc * HW;
  const int tid = threadIdx.x;
  {
    // all loads in flight before the first use (the map is read once; a strided
    // load-use loop would pay one HBM/L2 latency per iteration)
    constexpr int NL = kDecMaxHW / kDecThreads;
    float v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int i = tid + j * kDecThreads;
      v[j] = i < HW ? __builtin_nontemporal_load(src + i) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int i = tid + j * kDecThreads;
      if (i < HW) heat[i] = apply_sigmoid ? sigmoid_clamp_f(v[j]) : v[j];
    }
  }
  __syncthreads();
  // 3x3 peak test (F.max_pool2d(3, 1, 1) pads with -inf); threads own contiguous
  // index ranges so the tie scan below follows flat-index order.
  const int ipt = (HW + kDecThreads - 1) / kDecThreads;
  const int i0 = tid * ipt;
  const int i1 = min(i0 + ipt, HW);
  float pk[(kDecMaxHW + kDecThreads - 1) / kDecThreads];
  int y = i0 / W, x = i0 - (i0 / W) * W;  // walked incrementally (no per-item division)
#pragma unroll
  for (int j = 0; j < (kDecMaxHW + kDecThreads - 1) / kDecThreads; ++j) {
    const int i = i0 + j;
    float out = 0.f;
    if (i < i1) {
      const float v = heat[i];
      float m = v;
      for (int dy = -1; dy <= 1; ++dy) {
        const int yy = y + dy;
        if ((unsigned)yy >= (unsigned)H) continue;
        for (int dx = -1; dx <= 1; ++dx) {
          const int xx = x + dx;
          if ((unsigned)xx >= (unsigned)W) continue;
          m = fmaxf(m, heat[yy * W + xx]);
        }
      }
      out = (m == v) ? v : v * 0.f;  // heat * keep: non-peaks become (signed) zero
      if (++x == W) {
        x = 0;
        ++y;
      }
    }
    pk[j] = out;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < (kDecMaxHW + kDecThreads - 1) / kDecThreads; ++j)
    if (i0 + j < i1) heat[i0 + j] = pk[j];
  __syncthreads();

  // Radix select of the K-th largest key.
  unsigned prefix = 0u, pmask = 0u;
  int krem = K;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = tid; i < 256; i += kDecThreads) hist[i] = 0u;
    __syncthreads();
    // Non-peaks are exactly 0 (most of the map): count them per thread and add
    // them with one atomic per wave instead of hammering a single LDS bin.
    constexpr unsigned kZero = 0x80000000u;  // fkey(0.f)
    unsigned nzero = 0;
    for (int i = i0; i < i1; ++i) {
      const unsigned k = fkey(heat[i]);
      if ((k & pmask) == prefix) {
        if (k == kZero)
          ++nzero;
        else
          atomicAdd(&hist[(k >> shift) & 255u], 1u);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nzero += __shfl_xor(nzero, o, 64);
    if ((tid & 63) == 0 && nzero) atomicAdd(&hist[(kZero >> shift) & 255u], nzero);
    __syncthreads();
    if (tid < 64) {
      // descending suffix counts over 256 bins: lane handles bins 255-4*lane-3 .. 255-4*lane
      unsigned c4[4];
      unsigned loc = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        c4[q] = hist[255 - (4 * tid + q)];
        loc += c4[q];
      }
      unsigned x = loc;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(x, o, 64);
        if (tid >= o) x += y;
      }
      unsigned above = x - loc;  // keys in bins strictly above this lane's 4 bins
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (above < (unsigned)krem && above + c4[q] >= (unsigned)krem) {
          misc[0] = 255 - (4 * tid + q);
          misc[1] = krem - (int)above;
        }
        above += c4[q];
      }
    }
    __syncthreads();
    prefix |= (unsigned)misc[0] << shift;
    pmask |= 255u << shift;
    krem = misc[1];
    __syncthreads();
  }
  // prefix = exact key T of the K-th largest; krem = how many keys == T to take.
  const unsigned T = prefix;
  int nties = 0;
  for (int i = i0; i < i1; ++i) nties += fkey(heat[i]) == T;
  if (tid == 0) misc[2] = 0;
  const int tie_before = block_excl_scan(nties, wsum, nullptr);
  int tie_rank = tie_before;
  for (int i = i0; i < i1; ++i) {
    const unsigned k = fkey(heat[i]);
    bool take = k > T;
    if (k == T) {
      take = tie_rank < krem;
      ++tie_rank;
    }
    if (take) {
      const int slot = atomicAdd(&misc[2], 1);
      sel_key[slot] = k;
      sel_idx[slot] = i;
    }
  }
  __syncthreads();
  // rank the K selected entries: value desc, index asc
  if (tid < K) {
    const unsigned k = sel_key[tid];
    const int ix = sel_idx[tid];
    int rank = 0;
    for (int j = 0; j < K; ++j) {
      const unsigned kj = sel_key[j];
      rank += (kj > k) || (kj == k && sel_idx[j] < ix);
    }
    cand_key[(size_t)bc * K + rank] = k;
    cand_idx[(size_t)bc * K + rank] = ix;
  }
}

__global__ void __launch_bounds__(256) decode_merge_gather_kernel(
    const unsigned* __restrict__ cand_key, const int* __restrict__ cand_idx, int C, int K, int H,
    int W, int apply_sigmoid, const float* __restrict__ off, const float* __restrict__ dir,
    const float* __restrict__ z, const float* __restrict__ dim, float* __restrict__ dets) {
  __shared__ unsigned skey[16 * kDecMaxK];
  const int b = blockIdx.x;
  const int CK = C * K;
  const int HW = H * W;
  const unsigned* ck = cand_key + (size_t)b * CK;
  const int* ci = cand_idx + (size_t)b * CK;
  for (int t = threadIdx.x; t < CK; t += blockDim.x) skey[t] = ck[t];
  __syncthreads();
  for (int t = threadIdx.x; t < CK; t += blockDim.x) {
    const unsigned k = skey[t];
    int rank = 0;
    for (int j = 0; j < CK; ++j) {
      const unsigned kj = skey[j];
      rank += (kj > k) || (kj == k && j < t);
    }
    if (rank >= K) continue;
    const int cls = t / K;
    const int ind = ci[t];
    float xs = (float)(ind % W);
    float ys = (float)(ind / W);
    if (off) {
      float o0 = off[((size_t)b * 2 + 0) * HW + ind];
      float o1 = off[((size_t)b * 2 + 1) * HW + ind];
      if (apply_sigmoid) {
        o0 = sigmoid_clamp_f(o0);
        o1 = sigmoid_clamp_f(o1);
      }
      xs = xs + o0;
      ys = ys + o1;
    } else {
      xs = xs + 0.5f;
      ys = ys + 0.5f;
    }
    float* d = dets + ((size_t)b * K + rank) * 10;
    d[0] = fkey_inv(k);
    d[1] = xs;
    d[2] = ys;
    d[3] = z[(size_t)b * HW + ind];
    d[4] = dim[((size_t)b * 3 + 0) * HW + ind];
    d[5] = dim[((size_t)b * 3 + 1) * HW + ind];
    d[6] = dim[((size_t)b * 3 + 2) * HW + ind];
    d[7] = dir[((size_t)b * 2 + 0) * HW + ind];
    d[8] = dir[((size_t)b * 2 + 1) * HW + ind];
    d[9] = (float)cls;
  }
}

}  // namespace sfa

using namespace sfa;

extern "C" size_t sfa_decode_workspace_size(int batch, int num_classes, int K) {
  if (batch <= 0 || num_classes <= 0 || K <= 0) return 0;
  const size_t n = (size_t)batch * num_classes * K;
  return align_up(n * sizeof(unsigned), 256) + align_up(n * sizeof(int), 256);
}

extern "C" int sfa_decode(const float* hm, const float* off, const float* dir, const float* z,
                          const float* dim, int batch, int num_classes, int height, int width, int K,
                          int apply_sigmoid, float* dets, void* workspace, size_t workspace_bytes,
                          void* stream) {
  SFA_CHECK_ARG(hm && dir && z && dim && dets && workspace, "decode: null argument");
  SFA_CHECK_ARG(batch >= 1 && num_classes >= 1 && num_classes <= 16, "decode: bad B/C");
  SFA_CHECK_ARG(height >= 1 && width >= 1 && height * width <= kDecMaxHW,
                "decode: H*W = %d exceeds %d", height * width, kDecMaxHW);
  SFA_CHECK_ARG(K >= 1 && K <= kDecMaxK && K <= height * width, "decode: K = %d out of range", K);
  if (workspace_bytes < sfa_decode_workspace_size(batch, num_classes, K)) {
    set_error("decode: workspace too small");
    return SFA_E_WORKSPACE;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t n = (size_t)batch * num_classes * K;
  auto* ck = reinterpret_cast<unsigned*>(workspace);
  auto* ci = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) +
                                    align_up(n * sizeof(unsigned), 256));
  hipLaunchKernelGGL(decode_class_topk_kernel, dim3(batch * num_classes), dim3(kDecThreads), 0, st, hm, num_classes, height, width, K, apply_sigmoid, ck, ci);
  SFA_LAUNCH_CHECK();
  hipLaunchKernelGGL(decode_merge_gather_kernel, dim3(batch), dim3(256), 0, st, ck, ci,
                     num_classes, K, height, width, apply_sigmoid, off, dir, z, dim, dets);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}
