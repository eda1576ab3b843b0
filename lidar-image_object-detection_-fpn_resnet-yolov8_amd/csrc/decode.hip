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
//
// Round 3 — band-parallel form (the default whenever a band tile fits LDS): the 48 (frame,
// class) workgroups above left 208 of 256 CUs idle for ~60 us.  Now each class map is cut into
// S row bands (S = 8 at 152x152, K = 50: 384 workgroups of 256 threads), and
//   decode_band_topk_kernel: one workgroup per (band, class, frame) stages its R rows + a
//     1-row halo in LDS, applies sigmoid + clamp, runs the 3x3 peak test and selects the band's
//     top min(K, band) peaks by (value desc, index asc) with the same radix select + ordered
//     tie scan, written as a list sorted in that order (padded to K with sentinels);
//   decode_band_merge_gather_kernel: one workgroup per frame merges the C*S sorted band lists
//     pairwise in log2(C*S) rounds (each merge truncated to K) in (value desc, class asc,
//     index asc) order and gathers the K winners.
// Equivalence with the reference's two topk stages: an entry in the final top K has fewer than
// K entries before it in (value desc, class asc, index asc) order, hence fewer than K of its
// own class (or band) before it in that class's (value desc, index asc) order, so it survives
// every per-class (per-band) top-K; and torch's second stage orders equal values by class*K +
// rank = (class asc, index asc).  Same results bit for bit as the one-block-per-class kernels.
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

// PEAK = false: no 3x3 peak test (the reference's _topk / _topk_channel on a map as it is).
template <bool PEAK = true>
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
      if (PEAK) {
        for (int dy = -1; dy <= 1; ++dy) {
          const int yy = y + dy;
          if ((unsigned)yy >= (unsigned)H) continue;
          for (int dx = -1; dx <= 1; ++dx) {
            const int xx = x + dx;
            if ((unsigned)xx >= (unsigned)W) continue;
            m = fmaxf(m, heat[yy * W + xx]);
          }
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

constexpr int kBandThreads = 512;
constexpr int kBandWaves = kBandThreads / 64;
constexpr int kBandMaxTile = 8192;   // LDS floats of a band tile ((R + 2) x (W + 2), -inf border)
constexpr int kBandMaxIPT = 8;       // band pixels per thread
constexpr int kBandMaxLoads = 16;    // staged tile floats per thread
constexpr int kMergeMax = 4096;      // C * S * K candidates ranked per frame

// Block-wide exclusive scan of one int per thread (kBandWaves waves).
__device__ int band_excl_scan(int v, int* wsum /*[kBandWaves]*/) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int before = 0;
#pragma unroll
  for (int w = 0; w < kBandWaves; ++w) before += w < wave ? wsum[w] : 0;
  return before + x - v;
}

// ABL (timing ablations, tools/decodebench.hip only; results wrong): 1 = no sigmoid, 2 = no peak
// test, 4 = no radix select (nothing selected), 8 = no band sort
//
// grid (S, C, B): band s = rows [s*R, min(H, s*R + R)) of class map (b, c).  The band's rows
// plus a 1-row halo are staged in LDS with a -inf border (max_pool2d's padding: rows outside
// the map and columns -1 / W), so the 3x3 peak test is nine unconditional reads.  Writes the
// band's top min(K, band pixels) by (value desc, index asc) as a sorted list of K (key, index),
// padded with sentinels (key 0, index INT_MAX), to bkey / bidx[((b * C + c) * S + s) * K + j].
template <int ABL = 0, bool PEAK = true>
__global__ void __launch_bounds__(kBandThreads) decode_band_topk_kernel(
    const float* __restrict__ hm, int C, int H, int W, int K, int R, int apply_sigmoid,
    unsigned* __restrict__ bkey, int* __restrict__ bidx) {
  __shared__ __attribute__((aligned(16))) float tile[kBandMaxTile];
  __shared__ unsigned hist[256];
  __shared__ int wsum[kBandWaves];
  __shared__ int misc[4];
  __shared__ unsigned sel_key[kDecMaxK];
  __shared__ int sel_idx[kDecMaxK];
  const int s = blockIdx.x, c = blockIdx.y, b = blockIdx.z, S = gridDim.x;
  const int tid = threadIdx.x;
  const int y0 = s * R, y1 = min(H, y0 + R);
  const int TW = W + 2;                 // tile row: column -1, 0 .. W-1, W
  const int n_tile = (y1 - y0 + 2) * TW;  // tile rows y0 - 1 .. y1
  const float* src = hm + ((size_t)b * C + c) * H * W;
  {
    // every load in flight before the first use (the map is read once)
    float v[kBandMaxLoads];
#pragma unroll
    for (int j = 0; j < kBandMaxLoads; ++j) {
      const int i = tid + j * kBandThreads;
      const int r = i / TW, x = i - r * TW - 1, y = y0 - 1 + r;
      const bool in = i < n_tile && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      v[j] = in ? __builtin_nontemporal_load(src + (size_t)y * W + x) : -INFINITY;
    }
#pragma unroll
    for (int j = 0; j < kBandMaxLoads; ++j) {
      const int i = tid + j * kBandThreads;
      if (i < n_tile) {
        const int r = i / TW, x = i - r * TW - 1, y = y0 - 1 + r;
        const bool in = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;  // not the border
        tile[i] = (in && apply_sigmoid && !(ABL & 1)) ? sigmoid_clamp_f(v[j]) : v[j];
      }
    }
  }
  __syncthreads();
  // 3x3 peak test over the band's pixels; each thread owns a contiguous index range so the
  // tie scan follows flat-index order
  const int nb = (y1 - y0) * W;  // band pixels
  const int ipt = (nb + kBandThreads - 1) / kBandThreads;
  const int i0 = min(tid * ipt, nb), i1 = min(i0 + ipt, nb);
  unsigned key[kBandMaxIPT];
  {
    int r = i0 / W, x = i0 - (i0 / W) * W;  // band row, column (walked incrementally)
#pragma unroll
    for (int j = 0; j < kBandMaxIPT; ++j) {
      unsigned k = 0u;
      if (i0 + j < i1) {
        const float* t = tile + (r + 1) * TW + x + 1;  // the pixel; neighbours at +-1, +-TW
        const float v = t[0];
        float m = v;
        if (PEAK && !(ABL & 2)) {
          const float a0 = fmaxf(fmaxf(t[-TW - 1], t[-TW]), t[-TW + 1]);
          const float a1 = fmaxf(t[-1], t[1]);
          const float a2 = fmaxf(fmaxf(t[TW - 1], t[TW]), t[TW + 1]);
          m = fmaxf(m, fmaxf(a0, fmaxf(a1, a2)));
        }
        k = fkey((m == v) ? v : v * 0.f);  // heat * keep: non-peaks become (signed) zero
        if (++x == W) {
          x = 0;
          ++r;
        }
      }
      key[j] = k;
    }
  }
  const int kk = min(K, nb);  // real candidates of this band
  // Radix select of the kk-th largest key.
  unsigned prefix = (ABL & 4) ? 0xffffffffu : 0u, pmask = 0u;
  int krem = (ABL & 4) ? 0 : kk;
  for (int pass = 0; pass < ((ABL & 4) ? 0 : 4); ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = tid; i < 256; i += kBandThreads) hist[i] = 0u;
    __syncthreads();
    constexpr unsigned kZero = 0x80000000u;  // fkey(0.f): the non-peaks, counted per wave
    unsigned nzero = 0;
#pragma unroll
    for (int j = 0; j < kBandMaxIPT; ++j) {
      if (i0 + j < i1) {
        const unsigned k = key[j];
        if ((k & pmask) == prefix) {
          if (k == kZero)
            ++nzero;
          else
            atomicAdd(&hist[(k >> shift) & 255u], 1u);
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nzero += __shfl_xor(nzero, o, 64);
    if ((tid & 63) == 0 && nzero) atomicAdd(&hist[(kZero >> shift) & 255u], nzero);
    __syncthreads();
    if (tid < 64) {
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
      unsigned above = x - loc;
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
  const unsigned T = prefix;  // key of the kk-th largest; take krem of the keys == T
  int nties = 0;
#pragma unroll
  for (int j = 0; j < kBandMaxIPT; ++j)
    if (i0 + j < i1) nties += key[j] == T;
  if (tid == 0) misc[2] = 0;
  int tie_rank = band_excl_scan(nties, wsum);
  __syncthreads();  // misc[2] = 0 visible
  const int pix0 = y0 * W;  // flat index of the band's first pixel in the class map
#pragma unroll
  for (int j = 0; j < kBandMaxIPT; ++j) {
    if (i0 + j < i1) {
      const unsigned k = key[j];
      bool take = k > T;
      if (k == T) {
        take = tie_rank < krem;
        ++tie_rank;
      }
      if (take) {
        const int slot = atomicAdd(&misc[2], 1);
        sel_key[slot] = k;
        sel_idx[slot] = pix0 + i0 + j;
      }
    }
  }
  __syncthreads();
  // the band's list sorted by (value desc, index asc), then sentinels (key 0, index INT_MAX)
  // that never rank into the top K: the merge kernel merges these lists
  const size_t out0 = (((size_t)b * C + c) * S + s) * K;
  for (int t = tid; t < K; t += kBandThreads) {
    if (t < kk && !(ABL & 8)) {
      const unsigned k = sel_key[t];
      const int ix = sel_idx[t];
      int r0 = 0, r1 = 0, r2 = 0, r3 = 0;  // four independent chains (LDS latency)
      int j = 0;
      for (; j + 4 <= kk; j += 4) {
        const unsigned k0 = sel_key[j], k1 = sel_key[j + 1], k2 = sel_key[j + 2], k3 = sel_key[j + 3];
        const int x0 = sel_idx[j], x1 = sel_idx[j + 1], x2 = sel_idx[j + 2], x3 = sel_idx[j + 3];
        r0 += (k0 > k) || (k0 == k && x0 < ix);
        r1 += (k1 > k) || (k1 == k && x1 < ix);
        r2 += (k2 > k) || (k2 == k && x2 < ix);
        r3 += (k3 > k) || (k3 == k && x3 < ix);
      }
      for (; j < kk; ++j) r0 += (sel_key[j] > k) || (sel_key[j] == k && sel_idx[j] < ix);
      const int rank = r0 + r1 + r2 + r3;
      bkey[out0 + rank] = k;
      bidx[out0 + rank] = ix;
    } else {
      bkey[out0 + t] = 0u;
      bidx[out0 + t] = 0x7fffffff;
    }
  }
}

// One workgroup per frame: the C*S*K band candidates (L = C*S sorted lists of K) are merged
// pairwise, log2(L) rounds, each pair's merge truncated to its first K — the top K of a union
// of two lists comes from the top K of each — in (value desc, class asc, index asc) order: an
// entry's place in the merged pair is its own position plus the number of partner entries that
// precede it (a binary search; equal entries, only the sentinels, break left-first).  The K
// winners of the last list gather offset / direction / z / dim into (K, 10) rows
// (decode_merge_gather_kernel's columns).
__global__ void __launch_bounds__(1024) decode_band_merge_gather_kernel(
    const unsigned* __restrict__ bkey, const int* __restrict__ bidx, int C, int S, int K, int H,
    int W, int apply_sigmoid, const float* __restrict__ off, const float* __restrict__ dir,
    const float* __restrict__ z, const float* __restrict__ dim, float* __restrict__ dets) {
  __shared__ unsigned skey[2][kMergeMax];
  __shared__ int sidx[2][kMergeMax];  // class * 2^26 + index (index < 2^26 = the order within a key)
  const int b = blockIdx.x;
  const int SK = S * K, N = C * SK;
  const int HW = H * W;
  for (int t = threadIdx.x; t < N; t += blockDim.x) {
    const unsigned k = bkey[(size_t)b * N + t];
    const int ix = bidx[(size_t)b * N + t];
    skey[0][t] = k;
    sidx[0][t] = ix == 0x7fffffff ? 0x7fffffff : (t / SK) * (1 << 26) + ix;
  }
  __syncthreads();
  int cur = 0;
  for (int nl = C * S; nl > 1; nl = (nl + 1) >> 1) {
    const unsigned* ik = skey[cur];
    const int* ii = sidx[cur];
    unsigned* ok = skey[cur ^ 1];
    int* oi = sidx[cur ^ 1];
    for (int t = threadIdx.x; t < nl * K; t += blockDim.x) {
      const int l = t / K, p = t - l * K;
      const unsigned k = ik[t];
      const int ci = ii[t];
      int rank = p;
      if (!((nl & 1) && l == nl - 1)) {  // the odd list out is carried over as it is
        const bool left = (l & 1) == 0;
        const unsigned* pk = ik + (l ^ 1) * K;
        const int* pi = ii + (l ^ 1) * K;
        int lo = 0, hi = K;  // partner entries preceding (k, ci)
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          const unsigned km = pk[mid];
          const int im = pi[mid];
          const bool before = km > k || (km == k && (left ? im < ci : im <= ci));
          if (before)
            lo = mid + 1;
          else
            hi = mid;
        }
        rank += lo;
      }
      if (rank < K) {
        ok[(l >> 1) * K + rank] = k;
        oi[(l >> 1) * K + rank] = ci;
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  for (int rank = threadIdx.x; rank < K; rank += blockDim.x) {
    const unsigned k = skey[cur][rank];
    const int ci = sidx[cur][rank];
    const int cls = ci >> 26;
    const int ind = ci & ((1 << 26) - 1);
    if (ci == 0x7fffffff || ind >= HW || cls >= C) {  // a sentinel: unreachable while K <= H*W
      float* d = dets + ((size_t)b * K + rank) * 10;  // (sfa_decode checks it); never gathered
      for (int q = 0; q < 10; ++q) d[q] = 0.f;
      continue;
    }
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

// Band geometry: S bands of R rows (8 preferred: 384 workgroups at B = 16, C = 3) with
// C * S * K <= kMergeMax, (R + 2) * (W + 2) <= kBandMaxTile and ceil(R * W / 512) <= kBandMaxIPT;
// S = 0 when no band split fits (one block per class, the kernels above).
static void band_plan(int C, int H, int W, int K, int* S_out, int* R_out) {
  *S_out = 0;
  *R_out = H;
  static const int order[] = {8, 9, 10, 11, 12, 13, 14, 15, 16, 7, 6, 5, 4, 3, 2, 1};
  for (int S : order) {
    if (S > H) continue;
    const int R = (H + S - 1) / S;
    const int S_eff = (H + R - 1) / R;
    if (C * S_eff * K > kMergeMax) continue;
    if ((R + 2) * (W + 2) > kBandMaxTile || (R + 2) * (W + 2) > kBandMaxLoads * kBandThreads) continue;
    if ((R * W + kBandThreads - 1) / kBandThreads > kBandMaxIPT) continue;
    *S_out = S_eff;
    *R_out = R;
    return;
  }
}

// ---------------------------------------------------------------- helpers --
// The reference's decode helpers as device functions of their own (the drop-in
// utils.evaluation_utils serves them; VERDICT r03: no hot-path name may fall through to the
// reference's torch code).

// _nms (evaluation_utils.py:21-26): out = heat * (max_pool2d(heat, 3, 1, 1) == heat), the pool
// padded with -inf (neighbours outside the map are skipped), non-peaks (signed) zero like the
// float multiply. One thread per pixel; the nine reads hit L1 / L2 (out must not alias heat).
__global__ void __launch_bounds__(256) heat_nms_kernel(const float* __restrict__ heat, float* __restrict__ out,
                                                       int64_t n, int H, int W) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t HW = (int64_t)H * W;
  const int64_t p = i % HW;
  const int y = (int)(p / W), x = (int)(p - (int64_t)(p / W) * W);
  const float* map = heat + (i - p);
  const float v = heat[i];
  float m = v;
  for (int dy = -1; dy <= 1; ++dy) {
    const int yy = y + dy;
    if ((unsigned)yy >= (unsigned)H) continue;
    for (int dx = -1; dx <= 1; ++dx) {
      const int xx = x + dx;
      if ((unsigned)xx >= (unsigned)W) continue;
      m = fmaxf(m, map[(int64_t)yy * W + xx]);
    }
  }
  out[i] = (m == v) ? v : v * 0.f;
}

// _topk (:47-62, PERCH = false) / _topk_channel (:65-74, PERCH = true) outputs from the band
// lists of decode_band_topk_kernel<0, false> (no peak test). One workgroup per output group: a
// frame (its C * S lists, merged in (value desc, class asc, index asc) order = torch's second
// topk over class * K + rank), or a (frame, class) (its S lists: the class's own top K).  Columns
// as the reference computes them: score, ind (the flat index within the class map, int64),
// class (int32, PERCH = false), ys = floor(ind / W), xs = ind % W (floats).
template <bool PERCH>
__global__ void __launch_bounds__(1024) topk_band_merge_kernel(
    const unsigned* __restrict__ bkey, const int* __restrict__ bidx, int C, int S, int K, int W,
    float* __restrict__ out_score, int64_t* __restrict__ out_inds, int* __restrict__ out_cls,
    float* __restrict__ out_ys, float* __restrict__ out_xs) {
  __shared__ unsigned skey[2][kMergeMax];
  __shared__ int sidx[2][kMergeMax];  // class * 2^26 + index
  const int g = blockIdx.x;
  const int SK = S * K, N = PERCH ? SK : C * SK;
  for (int t = threadIdx.x; t < N; t += blockDim.x) {
    const unsigned k = bkey[(size_t)g * N + t];
    const int ix = bidx[(size_t)g * N + t];
    skey[0][t] = k;
    sidx[0][t] = ix == 0x7fffffff ? 0x7fffffff : (t / SK) * (1 << 26) + ix;
  }
  __syncthreads();
  int cur = 0;
  for (int nl = N / K; nl > 1; nl = (nl + 1) >> 1) {
    const unsigned* ik = skey[cur];
    const int* ii = sidx[cur];
    unsigned* ok = skey[cur ^ 1];
    int* oi = sidx[cur ^ 1];
    for (int t = threadIdx.x; t < nl * K; t += blockDim.x) {
      const int l = t / K, p = t - l * K;
      const unsigned k = ik[t];
      const int ci = ii[t];
      int rank = p;
      if (!((nl & 1) && l == nl - 1)) {
        const bool left = (l & 1) == 0;
        const unsigned* pk = ik + (l ^ 1) * K;
        const int* pi = ii + (l ^ 1) * K;
        int lo = 0, hi = K;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          const unsigned km = pk[mid];
          const int im = pi[mid];
          const bool before = km > k || (km == k && (left ? im < ci : im <= ci));
          if (before)
            lo = mid + 1;
          else
            hi = mid;
        }
        rank += lo;
      }
      if (rank < K) {
        ok[(l >> 1) * K + rank] = k;
        oi[(l >> 1) * K + rank] = ci;
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  for (int rank = threadIdx.x; rank < K; rank += blockDim.x) {
    const unsigned k = skey[cur][rank];
    const int ci = sidx[cur][rank];
    const int ind = ci & ((1 << 26) - 1);
    const size_t o = (size_t)g * K + rank;
    out_score[o] = fkey_inv(k);
    out_inds[o] = ind;
    if (!PERCH) out_cls[o] = ci >> 26;
    out_ys[o] = (float)(ind / W);
    out_xs[o] = (float)(ind % W);
  }
}

// The same outputs from the one-block-per-class candidates (decode_class_topk_kernel<false>:
// each class's K sorted by (value desc, index asc)) for maps whose bands do not fit LDS.
template <bool PERCH>
__global__ void __launch_bounds__(256) topk_class_out_kernel(
    const unsigned* __restrict__ cand_key, const int* __restrict__ cand_idx, int C, int K, int W,
    float* __restrict__ out_score, int64_t* __restrict__ out_inds, int* __restrict__ out_cls,
    float* __restrict__ out_ys, float* __restrict__ out_xs) {
  const int g = blockIdx.x;
  const int N = PERCH ? K : C * K;
  const unsigned* ck = cand_key + (size_t)g * N;
  const int* ci = cand_idx + (size_t)g * N;
  for (int t = threadIdx.x; t < N; t += blockDim.x) {
    const unsigned k = ck[t];
    int rank = t;
    if (!PERCH) {  // torch's second topk: value desc, then class * K + rank asc
      rank = 0;
      for (int j = 0; j < N; ++j) {
        const unsigned kj = ck[j];
        rank += (kj > k) || (kj == k && j < t);
      }
      if (rank >= K) continue;
    }
    const int ind = ci[t];
    const size_t o = (size_t)g * K + rank;
    out_score[o] = fkey_inv(k);
    out_inds[o] = ind;
    if (!PERCH) out_cls[o] = t / K;
    out_ys[o] = (float)(ind / W);
    out_xs[o] = (float)(ind % W);
  }
}

// _gather_feat (:29-37, mask None) and _transpose_and_gather_feat (:40-44): out[b][k][d] =
// feat[b * N * D + ind[b][k] * stride_n + d * stride_d] (elements of elem_bytes = 4 or 8:
// f32 / int32 features, or the int64 indices _topk gathers); indices checked by the caller.
template <typename T>
__global__ void __launch_bounds__(256) gather_feat_kernel(const T* __restrict__ feat, int64_t N, int D,
                                                          int64_t sn, int64_t sd, const int64_t* __restrict__ ind,
                                                          int K, int64_t total, T* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int d = (int)(i % D);
  const int64_t bk = i / D;
  const int64_t b = bk / K;
  out[i] = feat[b * N * D + ind[bk] * sn + (int64_t)d * sd];
}

}  // namespace sfa

using namespace sfa;

extern "C" size_t sfa_decode_workspace_size(int batch, int num_classes, int K) {
  if (batch <= 0 || num_classes <= 0 || K <= 0) return 0;
  // the band candidates (C * S * K per frame, S <= 16) or the per-class ones (C * K)
  const size_t n = (size_t)batch * num_classes * K * 16;
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
  int S = 0, R = height;
  band_plan(num_classes, height, width, K, &S, &R);
  if (S > 0) {
    const size_t nb = (size_t)batch * num_classes * S * K;
    auto* bk = reinterpret_cast<unsigned*>(workspace);
    auto* bi = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) + align_up(nb * sizeof(unsigned), 256));
    if (align_up(nb * sizeof(unsigned), 256) + nb * sizeof(int) > workspace_bytes) {
      set_error("decode: workspace too small");
      return SFA_E_WORKSPACE;
    }
    hipLaunchKernelGGL(decode_band_topk_kernel<0>, dim3(S, num_classes, batch), dim3(kBandThreads), 0, st, hm,
                       num_classes, height, width, K, R, apply_sigmoid, bk, bi);
    SFA_LAUNCH_CHECK();
    hipLaunchKernelGGL(decode_band_merge_gather_kernel, dim3(batch), dim3(1024), 0, st, bk, bi, num_classes, S,
                       K, height, width, apply_sigmoid, off, dir, z, dim, dets);
    SFA_LAUNCH_CHECK();
    return SFA_OK;
  }
  const size_t n = (size_t)batch * num_classes * K;
  auto* ck = reinterpret_cast<unsigned*>(workspace);
  auto* ci = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) +
                                    align_up(n * sizeof(unsigned), 256));
  hipLaunchKernelGGL(decode_class_topk_kernel<true>, dim3(batch * num_classes), dim3(kDecThreads), 0, st, hm, num_classes, height, width, K, apply_sigmoid, ck, ci);
  SFA_LAUNCH_CHECK();
  hipLaunchKernelGGL(decode_merge_gather_kernel, dim3(batch), dim3(256), 0, st, ck, ci,
                     num_classes, K, height, width, apply_sigmoid, off, dir, z, dim, dets);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

extern "C" int sfa_heat_nms(const float* heat, float* out, int64_t maps, int height, int width, void* stream) {
  SFA_CHECK_ARG(maps >= 0 && height >= 1 && width >= 1, "heat_nms: bad shape");
  const int64_t n = maps * (int64_t)height * width;
  if (n == 0) return SFA_OK;
  SFA_CHECK_ARG(heat && out && heat != out, "heat_nms: null or aliased buffers");
  hipLaunchKernelGGL(heat_nms_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), heat, out, n, height, width);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

extern "C" size_t sfa_topk_workspace_size(int batch, int num_classes, int K) {
  return sfa_decode_workspace_size(batch, num_classes, K);
}

extern "C" int sfa_topk(const float* scores, int batch, int num_classes, int height, int width, int K,
                        int per_channel, float* out_scores, int64_t* out_inds, int32_t* out_clses, float* out_ys,
                        float* out_xs, void* workspace, size_t workspace_bytes, void* stream) {
  SFA_CHECK_ARG(scores && out_scores && out_inds && out_ys && out_xs && workspace && (per_channel || out_clses),
                "topk: null argument");
  SFA_CHECK_ARG(batch >= 1 && num_classes >= 1 && num_classes <= 16, "topk: bad B/C");
  SFA_CHECK_ARG(height >= 1 && width >= 1 && height * width <= kDecMaxHW, "topk: H*W = %d exceeds %d",
                height * width, kDecMaxHW);
  SFA_CHECK_ARG(K >= 1 && K <= kDecMaxK && K <= height * width, "topk: K = %d out of range", K);
  if (workspace_bytes < sfa_topk_workspace_size(batch, num_classes, K)) {
    set_error("topk: workspace too small");
    return SFA_E_WORKSPACE;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int groups = per_channel ? batch * num_classes : batch;
  int S = 0, R = height;
  band_plan(num_classes, height, width, K, &S, &R);
  if (S > 0) {
    const size_t nb = (size_t)batch * num_classes * S * K;
    auto* bk = reinterpret_cast<unsigned*>(workspace);
    auto* bi = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) + align_up(nb * sizeof(unsigned), 256));
    hipLaunchKernelGGL((decode_band_topk_kernel<0, false>), dim3(S, num_classes, batch), dim3(kBandThreads), 0, st,
                       scores, num_classes, height, width, K, R, 0, bk, bi);
    SFA_LAUNCH_CHECK();
    if (per_channel)
      hipLaunchKernelGGL(topk_band_merge_kernel<true>, dim3(groups), dim3(1024), 0, st, bk, bi, num_classes, S, K,
                         width, out_scores, out_inds, out_clses, out_ys, out_xs);
    else
      hipLaunchKernelGGL(topk_band_merge_kernel<false>, dim3(groups), dim3(1024), 0, st, bk, bi, num_classes, S, K,
                         width, out_scores, out_inds, out_clses, out_ys, out_xs);
    SFA_LAUNCH_CHECK();
    return SFA_OK;
  }
  const size_t n = (size_t)batch * num_classes * K;
  auto* ck = reinterpret_cast<unsigned*>(workspace);
  auto* ci = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) + align_up(n * sizeof(unsigned), 256));
  hipLaunchKernelGGL(decode_class_topk_kernel<false>, dim3(batch * num_classes), dim3(kDecThreads), 0, st, scores,
                     num_classes, height, width, K, 0, ck, ci);
  SFA_LAUNCH_CHECK();
  if (per_channel)
    hipLaunchKernelGGL(topk_class_out_kernel<true>, dim3(groups), dim3(256), 0, st, ck, ci, num_classes, K, width,
                       out_scores, out_inds, out_clses, out_ys, out_xs);
  else
    hipLaunchKernelGGL(topk_class_out_kernel<false>, dim3(groups), dim3(256), 0, st, ck, ci, num_classes, K, width,
                       out_scores, out_inds, out_clses, out_ys, out_xs);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

extern "C" int sfa_gather_feat(const void* feat, int batch, int64_t n, int dim, int64_t stride_n, int64_t stride_d,
                               int elem_bytes, const int64_t* ind, int K, void* out, void* stream) {
  SFA_CHECK_ARG(batch >= 0 && n >= 1 && dim >= 1 && K >= 0 && (elem_bytes == 4 || elem_bytes == 8),
                "gather_feat: bad shape");
  const int64_t total = (int64_t)batch * K * dim;
  if (total == 0) return SFA_OK;
  SFA_CHECK_ARG(feat && ind && out, "gather_feat: null argument");
  const dim3 g((unsigned)((total + 255) / 256)), b(256);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (elem_bytes == 4)
    hipLaunchKernelGGL(gather_feat_kernel<unsigned>, g, b, 0, st, reinterpret_cast<const unsigned*>(feat), n, dim,
                       stride_n, stride_d, ind, K, total, reinterpret_cast<unsigned*>(out));
  else
    hipLaunchKernelGGL(gather_feat_kernel<unsigned long long>, g, b, 0, st,
                       reinterpret_cast<const unsigned long long*>(feat), n, dim, stride_n, stride_d, ind, K, total,
                       reinterpret_cast<unsigned long long*>(out));
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}
