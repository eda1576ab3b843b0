// Stem conv 7x7/s2/p3 (4 -> 64, NHWC4 input) + BN + ReLU + max-pool 3x3/s2/p1, fp16x3, from
// an LDS input patch (fpn_resnet.py:179-182).
//
// The implicit-GEMM stem (conv_h3_kernel<..., EPI_POOL>) gathers every K-tile of A from L2:
// 49 taps x 16 B per output pixel. Here a block instead stages, per 16 x 16 tile of the
// 304 x 304 conv output, the 37 x 38 input pixels its windows cover ONCE, split into two
// fp16 terms (x s = hi + lo, s the frame's power-of-two scale), and reads every MFMA A
// fragment from that patch. K is laid out (kh, kw 0..7, c 0..3) = 224 with a zero weight
// column at kw = 7, so the 8 k values a lane holds (two kw, four channels) are two adjacent
// patch pixels: one 16-B ds_read per term. The split weights (64 x 224 x 2 terms, 58 KiB)
// stay in LDS for the block's lifetime; blocks loop over tiles (grid = CUs) and prefetch
// the next tile's patch into registers while the current tile computes. Epilogue: the
// stem + pool epilogue of conv_h3_kernel (h3_pool_epilogue, 16 x 16 tiles).
//
// Round 3: the patch is read straight from the caller's layout (IN: NHWC4 from the voxeliser,
// or the reference's NCHW3 planes, optionally flipped for the back view), and each tile scales
// its patch by a power of two from ITS OWN max |x| (reduced over the prefetched patch while the
// previous tile computes) instead of the frame's: the layout-conversion pass (a 71 MB read +
// 95 MB write per 16 frames) and the input amax pass are gone.  A power-of-two scale only moves
// the fp16 terms' exponents, so products, f32 sums and the 1/s rescale give the same bits as
// the frame scale whenever the lo terms stay normal fp16 (|x| > 2^-16 of the scale's max; a
// tile's max is <= its frame's, so the tile scale is the more accurate one below that).
#pragma once

#include "conv_h3_kernel.h"

namespace sfa {

namespace stem_patch {
constexpr int TH = 16, TW = 16;                // conv-output tile
constexpr int PH = 2 * TH + 5, PW = 2 * TW + 6;  // patch: rows 2 oy - 3 + 0..36, cols 2 ox - 3 + 0..37
constexpr int PIX = PH * PW;                   // 1406
constexpr int KP = 224;                        // (kh, kw 0..7, c 0..3)
constexpr int WROW = KP * 2 + 16;              // bytes per W row in LDS (padded: conflict-free b128)
constexpr int W_BYTES = 2 * 64 * WROW;         // two fp16 terms
constexpr int PATCH_TERM = PIX * 8;            // 4 fp16 per pixel
constexpr int NT = 512, NW = 8;
constexpr int PF = (PIX + NT - 1) / NT;        // patch pixels prefetched per thread (3)
constexpr int T_BYTES = 256 * (64 + 4) * 4 + 2 * NW * 4;  // h3_pool_epilogue's LDS
constexpr int WM_BYTES = NW * 4;                             // per-wave max |x| of the next patch
constexpr int LDS_BYTES = W_BYTES + 2 * PATCH_TERM + T_BYTES + WM_BYTES;  // 151,632 B: one block per CU
}  // namespace stem_patch

// Epilogue for one 16 x 16 tile (th, tw) of frame b: ReLU(conv * 1/s * winv + b) into LDS,
// the frame's max recorded, then the 9 x 9 pooled cells whose 3 x 3/s2 window touches the
// tile (pooled rows 8 th .. 8 th + 8, cols 8 tw .. 8 tw + 8): each thread takes one cell and
// four channels, its window's nine float4 reads unrolled (indices clamped to the tile: a
// repeated element does not change a max).
// Default (a.part != null, no memset, no atomics): the tile stores the cells it owns (j, i <= 7:
// the cell's conv pixel (2 py, 2 px) lies in this tile) and writes its parts of the lower /
// right neighbours' cells (row j = 8, column i = 8) to its 17 side-buffer slots;
// stem_pool_merge_kernel folds those in. A/B form (a.part == null, SFA_STEM_PATCH_ATOMIC=1):
// cells with one writer (j, i in 1..7) are stored, the tile-border cells combined by
// atomicMax on the f32 bits (values >= +0) into the zeroed pooled buffer, as
// h3_pool_epilogue does. NOATOM (ablation ABL 16) applies to the A/B form only.
// ReLU(conv * 1/s * winv + b) of the wave's 32 rows into the tile T (row = 32 wave + q, q the
// row within the wave: pixel (2 wave + q / 16, q % 16)), returns the lane's max. One rounding
// (fmaf) per value, in both accumulator forms.
__device__ __forceinline__ float stem_tile_store32(const ConvArgs& a, x6_f32x16 (&acc)[1][2], float* T, int wave,
                                                   int tid, float ainv) {
  constexpr int LD = 68;
  const int lane = tid & 63, r = lane & 31, h = lane >> 5;
  float mx = 0.f;
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    const int n = ni * 32 + r;
    const float bn = a.bias[n];
    const float cs = a.winv[n] * ainv;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int row = wave * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
      float val = fmaf(acc[0][ni][v], cs, bn);
      val = val > 0.f ? val : 0.f;
      T[row * LD + n] = val;
      mx = fmaxf(mx, val);
    }
  }
  return mx;
}
// The same for the 16x16x32 form (acc[mi][ni]: lane l, register v -> row 16 mi + 4 (l >> 4) + v of
// the wave's 32, channel 16 ni + (l & 15); row stride 68 floats keeps the four row groups of a
// store on distinct banks).
__device__ __forceinline__ float stem_tile_store16(const ConvArgs& a, f32x4_t (&acc)[2][4], float* T, int wave, int tid,
                                                   float ainv) {
  constexpr int LD = 68;
  const int lane = tid & 63, c16 = lane & 15, g = lane >> 4;
  float mx = 0.f;
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = ni * 16 + c16;
    const float bn = a.bias[n];
    const float cs = a.winv[n] * ainv;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = wave * 32 + 16 * mi + 4 * g + v;
        float val = fmaf(acc[mi][ni][v], cs, bn);
        val = val > 0.f ? val : 0.f;
        T[row * LD + n] = val;
        mx = fmaxf(mx, val);
      }
  }
  return mx;
}

template <bool NOATOM = false>
__device__ __forceinline__ void stem_pool_epilogue(const ConvArgs& a, float mx, float* T, int b, int th, int tw,
                                                   int tid) {
  constexpr int LD = 68;
  if (a.amax_out)
    amax_commit_block<8>(a.amax_out, b, mx, 0.f, T + 256 * LD);  // includes __syncthreads
  else
    __syncthreads();
  const int PHo = a.OH >> 1, PWo = a.OW >> 1;
  const int c4 = tid & 15;
#pragma unroll
  for (int pass = 0; pass < 3; ++pass) {
    const int cell = (tid >> 4) + 32 * pass;
    if (cell >= 81) break;
    const int j = cell / 9, i = cell - 9 * j;
    const int py = 8 * th + j, px = 8 * tw + i;
    if (py >= PHo || px >= PWo) continue;
    const int ra = max(2 * j - 1, 0), rb = min(2 * j, 15), rc = min(2 * j + 1, 15);
    const int qa = max(2 * i - 1, 0), qb = min(2 * i, 15), qc = min(2 * i + 1, 15);
    const int rr[3] = {ra, rb, rc}, qq[3] = {qa, qb, qc};
    x6_f32x4 m = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int y = 0; y < 3; ++y)
#pragma unroll
      for (int x = 0; x < 3; ++x) {
        const x6_f32x4 t = *reinterpret_cast<const x6_f32x4*>(T + (rr[y] * 16 + qq[x]) * LD + 4 * c4);
#pragma unroll
        for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], t[e]);
      }
    float* dst = a.y + ((size_t)(b * PHo + py) * PWo + px) * 64 + 4 * c4;
    if (a.part) {  // side-buffer mode: cells j, i <= 7 are this tile's own, the rest go to its slots
      if (j <= 7 && i <= 7) {
        *reinterpret_cast<x6_f32x4*>(dst) = m;
      } else {
        const int slot = j == 8 ? i : 9 + j;
        const int tl = (b * (a.OH >> 4) + th) * (a.OW >> 4) + tw;
        *reinterpret_cast<x6_f32x4*>(a.part + ((size_t)tl * 17 + slot) * 64 + 4 * c4) = m;
      }
    } else if (NOATOM || (j >= 1 && j <= 7 && i >= 1 && i <= 7)) {
      *reinterpret_cast<x6_f32x4*>(dst) = m;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (m[e] > 0.f) atomicMax(reinterpret_cast<unsigned*>(dst) + e, __float_as_uint(m[e]));
    }
  }
}

// Side-buffer mode (a.part != null): every pooled cell has ONE owner tile, the tile holding
// conv pixel (2 py, 2 px); it stores its part of the window (rows/cols inside the tile) with a
// plain store. A tile's parts of its lower / right neighbours' cells (its pooled row j = 8 and
// column i = 8, 17 slots x 64 channels) go to a.part, and this kernel merges them into the
// owners' top-row / left-column cells: the up tile's row slot, the left tile's column slot,
// the up-left tile's corner slot — max is order-free, so the result equals the atomicMax form
// bit for bit, without 2,048 atomics per tile and without zeroing the pooled buffer first.
__global__ void __launch_bounds__(256) stem_pool_merge_kernel(const ConvArgs a, int frames) {
  const int tr = a.OH >> 4, tc = a.OW >> 4, PHo = a.OH >> 1, PWo = a.OW >> 1;
  const int per_tile = 15 * 16;  // 15 border cells (j = 0 row: i 0..7, i = 0 column: j 1..7) x 16 c4
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)frames * tr * tc * per_tile) return;
  const int c4 = (int)(idx & 15);
  const int e = (int)((idx >> 4) % 15);
  const int tl = (int)(idx / per_tile);
  const int b = tl / (tr * tc), t2 = tl - b * tr * tc, th = t2 / tc, tw = t2 - th * tc;
  const int j = e < 8 ? 0 : e - 7, i = e < 8 ? e : 0;
  const int py = 8 * th + j, px = 8 * tw + i;
  const bool up = j == 0 && th > 0, left = i == 0 && tw > 0;
  if (!up && !left) return;
  float* dst = a.y + ((size_t)(b * PHo + py) * PWo + px) * 64 + 4 * c4;
  x6_f32x4 m = *reinterpret_cast<const x6_f32x4*>(dst);
  auto merge = [&](int tile, int slot) {
    const x6_f32x4 t = *reinterpret_cast<const x6_f32x4*>(a.part + ((size_t)tile * 17 + slot) * 64 + 4 * c4);
#pragma unroll
    for (int q = 0; q < 4; ++q) m[q] = fmaxf(m[q], t[q]);
  };
  if (up) merge(tl - tc, i);
  if (left) merge(tl - 1, 9 + j);
  if (up && left) merge(tl - tc - 1, 8);
  *reinterpret_cast<x6_f32x4*>(dst) = m;
}

// The stem's split weights wh [2][64][Kpad] (k = (kh 7 + kw) 4 + c) -> LDS [2][64][WROW] at
// k' = (kh 8 + kw) 4 + c, the kw = 7 column zero: every load in flight before the first store (round 5:
// the load -> store loop waited one memory latency per iteration, 14 per block).
template <int NT, int WROW>
__device__ __forceinline__ void stem_stage_w(const ConvArgs& a, unsigned char* SW, int tid) {
  constexpr int ITEMS = 2 * 64 * 56, NWI = (ITEMS + NT - 1) / NT;
  // branch-free buffer loads: the kw = 7 column and the tail read out of range (zeros)
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.wh), (short)0,
                                                                       2 * 64 * a.Kpad * 2, 0x00020000);
  using u32x2 = unsigned __attribute__((ext_vector_type(2)));
  u32x2 wv[NWI];
#pragma unroll
  for (int j = 0; j < NWI; ++j) {
    const int i = tid + j * NT;
    const int t = i / (64 * 56), rem = i - t * (64 * 56);
    const int n = rem / 56, tap = rem - n * 56;
    const int kh = tap >> 3, kw = tap & 7;
    const unsigned off =
        i < ITEMS && kw < 7 ? (unsigned)(((t * 64 + n) * a.Kpad + (kh * 7 + kw) * 4) * 2) : 0x80000000u;
    wv[j] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rsw, off, 0, 0));
  }
#pragma unroll
  for (int j = 0; j < NWI; ++j) {
    const int i = tid + j * NT;
    const int t = i / (64 * 56), rem = i - t * (64 * 56);
    const int n = rem / 56, tap = rem - n * 56;
    if (i < ITEMS) *reinterpret_cast<u32x2*>(SW + t * 64 * WROW + n * WROW + tap * 8) = wv[j];
  }
}

// ABL (timing ablations only, env SFA_STEM_ABL; results wrong): 1 = no epilogue, 2 = no MFMAs,
// 4 = no patch fetch, 8 = first patch fetched after the weights are staged,
// 16 = border cells stored instead of atomicMax (only with a.part == null: the atomic A/B form),
// 64 = the 32x32x16 MFMA form (round 1) instead of 16x16x32 (same products, other summation order)
template <int ABL = 0, int IN = STEM_IN_NHWC4>
__global__ void __launch_bounds__(512, 1) stem_patch_pool_kernel(const ConvArgs a, int ntiles) {
  using namespace stem_patch;
  constexpr bool M16 = (ABL & 64) == 0;  // 16x16x32 MFMAs (default); ABL 64: the 32x32x16 form
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  unsigned char* SW = smem;
  unsigned char* SU = smem + W_BYTES;                   // patch, 2 terms
  unsigned char* ST = smem + W_BYTES + 2 * PATCH_TERM;  // epilogue tile (its own LDS: no barrier
                                                        // between a tile's epilogue and the next patch)
  float* WM = reinterpret_cast<float*>(smem + W_BYTES + 2 * PATCH_TERM + T_BYTES);
  // LDS-only barrier (the no-return pooled atomics of the previous tile stay in flight)
  auto lds_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  const ConvSeg& g = a.seg[0];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tw_n = a.OW / TW, tiles_per_frame = (a.OH / TH) * tw_n;

  // two patch prefetch sets: tile t's patch is loaded two tiles ahead (set t & 1), so the loads
  // have a whole tile (MFMAs + epilogue) to land before its max and split are needed
  x6_f32x4 pf0[PF], pf1[PF];
  auto fetch = [&](int tile, x6_f32x4 (&pf)[PF]) {
    const int b = tile / tiles_per_frame, tl = tile - b * tiles_per_frame;
    const int th = tl / tw_n, tw = tl - th * tw_n;
    const int iy0 = 2 * TH * th - 3, ix0 = 2 * TW * tw - 3;
    const size_t hw = (size_t)g.H * g.W;
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int p = tid + j * NT;
      const int py = p / PW, px = p - py * PW;
      const int iy = iy0 + py, ix = ix0 + px;
      x6_f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (p < PIX && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W) {
        if constexpr (IN == STEM_IN_NHWC4) {
          v = reinterpret_cast<const x6_f32x4*>(g.x)[(size_t)b * hw + iy * g.W + ix];
        } else {  // the reference's (B, 3, H, W) planes; channel 3 of the patch pixel stays 0
          const int sy = IN == STEM_IN_NCHW3_FLIP ? g.H - 1 - iy : iy;
          const int sx = IN == STEM_IN_NCHW3_FLIP ? g.W - 1 - ix : ix;
          const float* x = g.x + (size_t)b * 3 * hw + (size_t)sy * g.W + sx;
          v[0] = x[0];
          v[1] = x[hw];
          v[2] = x[2 * hw];
        }
      }
      pf[j] = v;
    }
  };
  // max |x| of the prefetched patch: this wave's part into WM (read after the next barrier)
  auto patch_max_to_lds = [&](const x6_f32x4 (&pf)[PF]) {
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < PF; ++j)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(pf[j][0]), fabsf(pf[j][1])), fmaxf(fabsf(pf[j][2]), fabsf(pf[j][3]))));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) WM[wave] = m;
  };
  auto store_patch = [&](float s, const x6_f32x4 (&pf)[PF]) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int p = tid + j * NT;
      if (p < PIX) {
        f16x4_t hi, lo;
        split2h(pf[j], s, hi, lo);
        *reinterpret_cast<f16x4_t*>(SU + p * 8) = hi;
        *reinterpret_cast<f16x4_t*>(SU + PATCH_TERM + p * 8) = lo;
      }
    }
  };

  const int r = lane & 31, h = lane >> 5;
  // A fragment origin of this lane: conv-output pixel (oy, ox) = (2 wave + r / 16, r % 16) of the
  // tile -> patch pixel (2 oy, 2 ox) + (kh, 4 (s & 1) + 2 h) at k-step s
  const int oyl = 2 * wave + (r >> 4), oxl = r & 15;
  const int abase = ((2 * oyl) * PW + 2 * oxl + 2 * h) * 8;
  const int bbase = r * WROW + 16 * h;

  const int G = gridDim.x;
  int tile = blockIdx.x;
  if (!(ABL & 4) && !(ABL & 8)) {  // in flight while the weights are staged
    if (tile < ntiles) fetch(tile, pf0);
    if (tile + G < ntiles) fetch(tile + G, pf1);
  }
  // weights: wh [2][64][Kpad] with k = (kh 7 + kw) 4 + c  ->  LDS [2][64][WROW] at k' = (kh 8 + kw) 4 + c
  stem_stage_w<NT, WROW>(a, SW, tid);

  if (!(ABL & 4) && (ABL & 8)) {
    if (tile < ntiles) fetch(tile, pf0);
    if (tile + G < ntiles) fetch(tile + G, pf1);
  }
  if (tile < ntiles) patch_max_to_lds(pf0);
  // one tile: patch `cur` (its max already in WM) split into LDS, the tile two ahead fetched into
  // `cur`, MFMAs, epilogue, then the max of `nxt` (the next tile's patch) into WM
  auto body = [&](int tile, x6_f32x4 (&cur)[PF], x6_f32x4 (&nxt)[PF]) {
    // WM of this patch visible (written after the previous tile's epilogue); first time round
    // also the staged weights
    __syncthreads();
    const int b = tile / tiles_per_frame;
    float ainv[1];
    float tmax = WM[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) tmax = fmaxf(tmax, WM[w]);
    const float as = amax_scale_bits(__float_as_uint(tmax), ainv[0]);
    store_patch(as, cur);
    // patch (and, first time round, the weights) in LDS; every wave is past the previous
    // tile's epilogue reads of ST
    lds_barrier();
    if (tile + 2 * G < ntiles && !(ABL & 4)) fetch(tile + 2 * G, cur);  // lands during the next tile

    float mx;
    if constexpr (M16) {
      // 16x16x32: k-step s = kh (32 k = kw 0..7 x c 0..3); lane (row l & 15, k-group g = l >> 4)
      // holds kw 2g, 2g + 1 of its row's pixel = one 16-B patch read per term; 2 row blocks
      // (conv rows 2 wave, 2 wave + 1) x 4 column blocks x 3 products per k-step
      f32x4_t acc[2][4];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int c16 = lane & 15, g4 = lane >> 4;
      const int abase16 = ((2 * (2 * wave)) * PW + 2 * c16 + 2 * g4) * 8;  // row block 0: conv row 2 wave
      const int bbase16 = c16 * WROW + 16 * g4;
#pragma unroll
      for (int s = 0; s < ((ABL & 2) ? 0 : KP / 32); ++s) {
        f16x8_t ahi[2], alo[2];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          const int aoff = abase16 + (2 * mi * PW + s * PW) * 8;  // conv row + mi -> patch row + 2 mi
          ahi[mi] = *reinterpret_cast<const f16x8_t*>(SU + aoff);
          alo[mi] = *reinterpret_cast<const f16x8_t*>(SU + PATCH_TERM + aoff);
        }
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const unsigned char* wb = SW + bbase16 + ni * 16 * WROW + 64 * s;
          const f16x8_t whi = *reinterpret_cast<const f16x8_t*>(wb);
          const f16x8_t wlo = *reinterpret_cast<const f16x8_t*>(wb + 64 * WROW);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) {
            f32x4_t cc = acc[mi][ni];
            cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[mi], whi, cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[mi], wlo, cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[mi], whi, cc, 0, 0, 0);
            acc[mi][ni] = cc;
          }
        }
      }
      mx = stem_tile_store16(a, acc, reinterpret_cast<float*>(ST), wave, tid, ainv[0]);
    } else {
      x6_f32x16 acc[1][2];
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[0][ni][v] = 0.f;
#pragma unroll
      for (int s = 0; s < ((ABL & 2) ? 0 : KP / 16); ++s) {
        const int aoff = abase + ((s >> 1) * PW + 4 * (s & 1)) * 8;
        const f16x8_t ahi = *reinterpret_cast<const f16x8_t*>(SU + aoff);
        const f16x8_t alo = *reinterpret_cast<const f16x8_t*>(SU + PATCH_TERM + aoff);
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const unsigned char* wb = SW + bbase + ni * 32 * WROW + 32 * s;
          const f16x8_t whi = *reinterpret_cast<const f16x8_t*>(wb);
          const f16x8_t wlo = *reinterpret_cast<const f16x8_t*>(wb + 64 * WROW);
          x6_f32x16 cc = acc[0][ni];
          cc = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, whi, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, wlo, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ahi, whi, cc, 0, 0, 0);
          acc[0][ni] = cc;
        }
      }
      mx = stem_tile_store32(a, acc, reinterpret_cast<float*>(ST), wave, tid, ainv[0]);
    }
    // the epilogue's own barrier (after its ST writes) also orders this tile's patch reads
    // before the next tile's patch stores
    if constexpr ((ABL & 1) != 0) {
      if (mx == 1234.5f) a.y[tid] = mx;
      __syncthreads();
    } else {
      const int tl = tile - b * tiles_per_frame, th = tl / tw_n;
      stem_pool_epilogue<(ABL & 16) != 0>(a, mx, reinterpret_cast<float*>(ST), b, th, tl - th * tw_n, tid);
    }
    // the next patch's max into WM (every wave read WM before this tile's lds_barrier)
    if (tile + G < ntiles) patch_max_to_lds(nxt);
  };
  for (;;) {
    if (tile >= ntiles) break;
    body(tile, pf0, pf1);
    tile += G;
    if (tile >= ntiles) break;
    body(tile, pf1, pf0);
    tile += G;
  }
}

// Round 3b: the same conv, scales and pool, one barrier per tile (stem_patch_pool_kernel has
// three), the pool computed from the accumulators instead of a 64 KiB LDS image of the tile.
//  * Patches double-buffered in LDS: tile t's MFMAs read patch buffer t & 1 while the split of
//    tile t + G's patch (its max reduced before the previous barrier) goes to the other one.
//  * Pool: lane (c, g) of a wave holds conv columns 4g .. 4g + 3 of rows 2w, 2w + 1 for channels
//    16 ni + c. Horizontal 3-maxima of the pooled columns 2g, 2g + 1 (and 8 for g = 3) come from
//    the lane's own values and column 4g - 1 of lane l - 16 (one bpermute per value); the vertical
//    3-maximum of pooled row w needs conv row 2w - 1, wave w - 1's second row: every wave
//    publishes its second row's horizontal maxima (9 x 64 floats) in an exchange buffer, and
//    after the tile's barrier each wave finishes its pooled row from registers + that buffer
//    (wave 7 also the row-8 partials). Ownership, side-buffer slots and the merge pass are
//    stem_pool_epilogue's (side-buffer mode only); the values are the same maxima of the same
//    ReLU(fmaf(acc, winv / s, b)) values: bit-identical output.
//  * Per tile, between barriers: the previous tile's pooled row (stores), the next patch's split,
//    this tile's MFMAs, its ReLU / horizontal maxima / exchange writes, the max of the patch two
//    ahead. ABL 1: waves 4-7 issue their MFMAs first and the previous tile's stores and the split
//    after them, so the two waves of a SIMD do not reach their MFMAs together.
namespace stem_patch2 {
using namespace stem_patch;
constexpr int XCH_W = 9 * 64 * 4;                  // one wave's second-row horizontal maxima
constexpr int XCH_BYTES = NW * XCH_W;              // per buffer
// + the output channels' winv / bias (round 5: read from LDS in the epilogue instead of 8 global loads
// per tile, which hipcc issued as four dependent round trips)
constexpr int LDS2 = W_BYTES + 2 * 2 * PATCH_TERM + 2 * XCH_BYTES + 2 * 2 * NW * 4 + 2 * 64 * 4;  // 141,888 B
}  // namespace stem_patch2

template <int IN = STEM_IN_NHWC4, int ABL = 0>
__global__ void __launch_bounds__(512, 1) stem_patch_pool2_kernel(const ConvArgs a, int ntiles) {
#pragma clang fp contract(off)
  using namespace stem_patch2;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS2];
  unsigned char* SW = smem;
  unsigned char* SU0 = smem + W_BYTES;                              // patch buffers: [2][2 terms]
  float* XCH0 = reinterpret_cast<float*>(SU0 + 4 * PATCH_TERM);      // [2][NW][9][64]
  float* WMX = XCH0 + 2 * XCH_BYTES / 4;                             // [2][NW] patch maxima
  float* TMX = WMX + 2 * NW;                                         // [2][NW] tile (ReLU) maxima
  float* CSB = TMX + 2 * NW;                                         // [64] winv, [64] bias
  const ConvSeg& g = a.seg[0];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tw_n = a.OW / TW, tiles_per_frame = (a.OH / TH) * tw_n;
  const int PHo = a.OH >> 1, PWo = a.OW >> 1;

  // Patch fetch. NHWC4: thread p loads patch pixels p, p + 512, p + 1024 (one float4 each).
  // NCHW3 (and flipped): item p < 370 = (patch row p / 10, column group p % 10) loads columns
  // 32 tw - 4 + 4 q .. + 3 of that row from each of the three planes as one aligned float4 (W % 4
  // == 0: a group lies wholly inside or wholly outside the image), i.e. patch columns 4 q - 1 ..
  // 4 q + 2 (column -1 is dropped): 3 loads per item instead of 3 per pixel.
  constexpr bool VEC = IN != STEM_IN_NHWC4;
  constexpr int NG = (PW + 1 + 3) / 4;  // column groups per patch row: 10
  static_assert(!VEC || PH * NG <= NT, "one item per thread");
  x6_f32x4 R0[PF], R1[PF];
  // branch-free buffer loads (out-of-range offsets read zeros): no zeroing of the patch registers
  // ahead of a conditional load, which made hipcc wait for every outstanding store first (round 5)
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(g.x), (short)0,
      (int)((size_t)(ntiles / tiles_per_frame) * (VEC ? 3 : 4) * g.H * g.W * 4), 0x00020000);
  auto fetch = [&](int tile, x6_f32x4 (&pf)[PF]) {
    const int b = tile / tiles_per_frame, tl = tile - b * tiles_per_frame;
    const int th = tl / tw_n, tw = tl - th * tw_n;
    const int iy0 = 2 * TH * th - 3, ix0 = 2 * TW * tw - 3;
    const size_t hw = (size_t)g.H * g.W;
    if constexpr (VEC) {
      const int py = tid / NG, q = tid - py * NG;
      const int iy = iy0 + py, ixg = ix0 - 1 + 4 * q;
      const bool ok = py < PH && (unsigned)iy < (unsigned)g.H && (unsigned)ixg < (unsigned)g.W;
      const int sy = IN == STEM_IN_NCHW3_FLIP ? g.H - 1 - iy : iy;
      const int sx = IN == STEM_IN_NCHW3_FLIP ? g.W - 4 - ixg : ixg;
      const unsigned base = (unsigned)(((size_t)b * 3 * hw + (size_t)sy * g.W + sx) * 4);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const x6_f32x4 v = __builtin_bit_cast(
            x6_f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsx, ok ? base + (unsigned)(c * hw * 4) : 0x80000000u, 0, 0));
        pf[c] = IN == STEM_IN_NCHW3_FLIP ? x6_f32x4{v[3], v[2], v[1], v[0]} : v;
      }
    } else {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int p = tid + j * NT;
        const int py = p / PW, px = p - py * PW;
        const int iy = iy0 + py, ix = ix0 + px;
        const bool ok = p < PIX && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
        pf[j] = __builtin_bit_cast(x6_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rsx, ok ? (unsigned)(((size_t)b * hw + iy * g.W + ix) * 16) : 0x80000000u, 0, 0));
      }
    }
  };
  auto patch_max = [&](const x6_f32x4 (&pf)[PF], float* dst) {
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < PF; ++j)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(pf[j][0]), fabsf(pf[j][1])), fmaxf(fabsf(pf[j][2]), fabsf(pf[j][3]))));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) dst[wave] = m;
  };
  // scale of a patch from its published per-wave maxima; split into patch buffer SU
  auto split_patch = [&](const float* wm, const x6_f32x4 (&pf)[PF], unsigned char* SU) -> float {
    float tmax = wm[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) tmax = fmaxf(tmax, wm[w]);
    float ainv;
    const float s = amax_scale_bits(__float_as_uint(tmax), ainv);
    if constexpr (VEC) {
      const int py = tid / NG, q = tid - py * NG;
      if (py < PH) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int px = 4 * q - 1 + e;
          if (px >= 0 && px < PW) {
            f16x4_t hi, lo;
            split2h(x6_f32x4{pf[0][e], pf[1][e], pf[2][e], 0.f}, s, hi, lo);
            *reinterpret_cast<f16x4_t*>(SU + (py * PW + px) * 8) = hi;
            *reinterpret_cast<f16x4_t*>(SU + PATCH_TERM + (py * PW + px) * 8) = lo;
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int p = tid + j * NT;
        if (p < PIX) {
          f16x4_t hi, lo;
          split2h(pf[j], s, hi, lo);
          *reinterpret_cast<f16x4_t*>(SU + p * 8) = hi;
          *reinterpret_cast<f16x4_t*>(SU + PATCH_TERM + p * 8) = lo;
        }
      }
    }
    return ainv;
  };

  const int G = gridDim.x;
  // logical block: consecutive tiles (row neighbours, whose patches share 5 input columns and the
  // 128-B lines of each patch row) on one XCD at the same time, so its L2 serves the shared lines once
  // (round 6: in blockIdx order neighbours ran on different XCDs)
  const int t0 = xcd_remap(blockIdx.x, G);
  if (t0 < ntiles) fetch(t0, R0);
  if (t0 + G < ntiles) fetch(t0 + G, R1);
  // weights: wh [2][64][Kpad], k = (kh 7 + kw) 4 + c  ->  LDS [2][64][WROW] at k' = (kh 8 + kw) 4 + c
  stem_stage_w<NT, WROW>(a, SW, tid);
  if (tid < 64) {  // published by the first tile's barriers
    const float wv = a.winv[tid], bv = a.bias[tid];
    CSB[tid] = wv;
    CSB[64 + tid] = bv;
  }
  if (t0 >= ntiles) return;  // uniform per block
  patch_max(R0, WMX);
  __syncthreads();
  float ainv_cur = split_patch(WMX, R0, SU0);
  if (t0 + 2 * G < ntiles) fetch(t0 + 2 * G, R0);
  if (t0 + G < ntiles) patch_max(R1, WMX + NW);
  __syncthreads();

  const int c16 = lane & 15, g4 = lane >> 4;
  const int abase16 = ((2 * (2 * wave)) * PW + 2 * c16 + 2 * g4) * 8;
  const int bbase16 = c16 * WROW + 16 * g4;
  // the previous tile's horizontal maxima: [mi][ni][k], k = pooled column 2 g4, 2 g4 + 1, 8 (g4 = 3)
  float hp[2][4][3];
  int prev_tile = -1;

  auto finish_prev = [&](int par) {  // vertical maxima + stores of tile prev_tile (exchange buffer par)
    if (prev_tile < 0) return;
    const int b = prev_tile / tiles_per_frame, tl = prev_tile - b * tiles_per_frame;
    const int th = tl / tw_n, tw = tl - th * tw_n;
    const float* X = XCH0 + par * (XCH_BYTES / 4);
    const int tlg = (b * (a.OH >> 4) + th) * (a.OW >> 4) + tw;  // side-buffer tile index
    const int py = 8 * th + wave;                                // pooled row j = wave
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int n = ni * 16 + c16;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (k == 2 && g4 != 3) continue;
        const int i = k == 2 ? 8 : 2 * g4 + k;
        float v = fmaxf(hp[0][ni][k], hp[1][ni][k]);
        if (wave > 0) v = fmaxf(v, X[((wave - 1) * 9 + i) * 64 + n]);
        const int px = 8 * tw + i;
        if (py < PHo && px < PWo) {
          if (i <= 7)
            a.y[((size_t)(b * PHo + py) * PWo + px) * 64 + n] = v;
          else
            a.part[((size_t)tlg * 17 + 9 + wave) * 64 + n] = v;
        }
        if (wave == NW - 1) {  // pooled row 8: conv row 15 only -> the lower neighbour's slot i
          const int py8 = 8 * th + 8;
          if (py8 < PHo && px < PWo) a.part[((size_t)tlg * 17 + i) * 64 + n] = hp[1][ni][k];
        }
      }
    }
    if (tid == 0 && a.amax_out) {
      const float* tm = TMX + par * NW;
      float m = tm[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) m = fmaxf(m, tm[w]);
      if (m > 0.f) amax_atomic(a.amax_out, b, m);
    }
  };

  // one tile; PAR = its parity (patch buffer, exchange buffer, maxima slots). Rs holds the next
  // tile's patch (split now, then refilled with the patch three tiles ahead), Rm the patch two
  // tiles ahead (its max reduced at the end). Compile-time parity keeps both sets in registers.
  auto body = [&](auto par_c, int tile, x6_f32x4 (&Rs)[PF], x6_f32x4 (&Rm)[PF]) {
    constexpr int par = decltype(par_c)::value;
    unsigned char* SUc = SU0 + par * 2 * PATCH_TERM;
    unsigned char* SUn = SU0 + (par ^ 1) * 2 * PATCH_TERM;
    const bool has_next = tile + G < ntiles;
    float ainv_next = 0.f;
    auto prep_next = [&]() {  // the next tile's patch into the other buffer; refill its registers
      if (!has_next) return;
      ainv_next = split_patch(WMX + (par ^ 1) * NW, Rs, SUn);
      if (tile + 3 * G < ntiles) fetch(tile + 3 * G, Rs);
    };
    const bool late = (ABL & 1) != 0 && wave >= NW / 2;
    if (!late) {
      finish_prev(par ^ 1);
      prep_next();
    }
    // MFMAs (stem_patch_pool_kernel's 16x16x32 form)
    f32x4_t acc[2][4];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KP / 32; ++s) {
      f16x8_t ahi[2], alo[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const int aoff = abase16 + (2 * mi * PW + s * PW) * 8;
        ahi[mi] = *reinterpret_cast<const f16x8_t*>(SUc + aoff);
        alo[mi] = *reinterpret_cast<const f16x8_t*>(SUc + PATCH_TERM + aoff);
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const unsigned char* wb = SW + bbase16 + ni * 16 * WROW + 64 * s;
        const f16x8_t whi = *reinterpret_cast<const f16x8_t*>(wb);
        const f16x8_t wlo = *reinterpret_cast<const f16x8_t*>(wb + 64 * WROW);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          f32x4_t cc = acc[mi][ni];
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[mi], whi, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[mi], wlo, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[mi], whi, cc, 0, 0, 0);
          acc[mi][ni] = cc;
        }
      }
    }
    if (late) {
      finish_prev(par ^ 1);
      prep_next();
    }
    // ReLU(conv * winv / s + b); horizontal maxima; the second row's into the exchange buffer
    float mx = 0.f;
    float* X = XCH0 + par * (XCH_BYTES / 4) + wave * 9 * 64;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int n = ni * 16 + c16;
      const float bn = CSB[64 + n];
      const float cs = CSB[n] * ainv_cur;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float t = fmaf(acc[mi][ni][e], cs, bn);
          v[e] = t > 0.f ? t : 0.f;
          mx = fmaxf(mx, v[e]);
        }
        const float left = __shfl_up(v[3], 16, 64);  // column 4 g4 - 1 (lane l - 16); unused for g4 = 0
        hp[mi][ni][0] = g4 > 0 ? fmaxf(fmaxf(left, v[0]), v[1]) : fmaxf(v[0], v[1]);
        hp[mi][ni][1] = fmaxf(fmaxf(v[1], v[2]), v[3]);
        hp[mi][ni][2] = v[3];
        if (mi == 1) {
          X[(2 * g4) * 64 + n] = hp[1][ni][0];
          X[(2 * g4 + 1) * 64 + n] = hp[1][ni][1];
          if (g4 == 3) X[8 * 64 + n] = v[3];
        }
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if (lane == 0) TMX[par * NW + wave] = mx;
    // the max of the patch two tiles ahead (its registers were refilled during the previous tile)
    if (tile + 2 * G < ntiles) patch_max(Rm, WMX + par * NW);
    prev_tile = tile;
    ainv_cur = ainv_next;
    __syncthreads();
  };
  int k = 0;
  for (int tile = t0;;) {
    if (tile >= ntiles) break;
    body(std::integral_constant<int, 0>(), tile, R1, R0);
    tile += G;
    ++k;
    if (tile >= ntiles) break;
    body(std::integral_constant<int, 1>(), tile, R0, R1);
    tile += G;
    ++k;
  }
  finish_prev((k - 1) & 1);
}

// Grid = one block per CU (each loops over tiles); needs the stem's fp16x3 split weights
// (Kpad >= 196), the input as a.stem_in says (seg 0 describes it as 4 channels), conv output
// divisible into 16 x 16 tiles.
inline int launch_stem_patch_pool(const ConvArgs& a, hipStream_t st) {
  const ConvSeg& g = a.seg[0];
  if (!a.wh || !a.winv || a.nseg != 1 || a.N != 64 || g.C != 4 || g.KH != 7 || g.KW != 7 || g.stride != 2 ||
      g.pad != 3 || a.Kpad < 196 || a.OH % 16 != 0 || a.OW % 16 != 0 || a.OH * 2 != g.H || a.OW * 2 != g.W ||
      a.res || !a.relu || (a.part && a.part_floats < (size_t)a.M / 256 * 17 * 64)) {
    set_error("stem_patch: unsupported stem (C=%d k=%d OH=%d OW=%d)", g.C, g.KH, a.OH, a.OW);
    return SFA_E_UNSUPPORTED;
  }
  const int frames = a.M / (a.OH * a.OW);
  const int ntiles = frames * (a.OH / 16) * (a.OW / 16);
  const int ncu = cu_count(st);
  const int grid = ntiles < ncu ? ntiles : ncu;
  if (grid <= 0) return SFA_OK;
  const dim3 gd((unsigned)grid), bd(stem_patch::NT);
  // the one-barrier kernel with waves 4-7 issuing their MFMAs first (it reads NCHW3 planes as
  // aligned float4 column groups); an NCHW3 input that is not 16-B aligned takes the round-3a
  // three-barrier kernel (4-B plane reads). The timing ablations and the rejected variants live in
  // tools/experiments/r03/stem_patch_kernel.h.
  const bool al16 = (reinterpret_cast<uintptr_t>(a.seg[0].x) & 15) == 0;
  if (!a.part) {
    set_error("stem_patch: the pooled tile-border parts need the side buffer (a.part)");
    return SFA_E_INVALID;
  }
  if (al16 || a.stem_in == STEM_IN_NHWC4) {
    // the kernel reads the input through a buffer resource with 32-bit offsets: batches whose input
    // reaches 2 GiB run in frame chunks (the side-buffer slots keep their global tile index)
    const size_t fbytes = (size_t)(a.stem_in == STEM_IN_NHWC4 ? 4 : 3) * g.H * g.W * 4;
    const int fchunk = (int)std::min<size_t>((size_t)frames, ((1ull << 31) - 1) / fbytes);
    if (fchunk < 1) {
      set_error("stem_patch: one %d x %d frame exceeds the 32-bit buffer offsets", g.H, g.W);
      return SFA_E_UNSUPPORTED;
    }
    const int tpf = (a.OH / 16) * (a.OW / 16);
    for (int f0 = 0; f0 < frames; f0 += fchunk) {
      const int nf = std::min(fchunk, frames - f0);
      ConvArgs c = a;
      c.seg[0].x = g.x + (size_t)f0 * (fbytes / 4);
      c.seg[0].bytes = (size_t)nf * fbytes;
      c.y = a.y + (size_t)f0 * (a.OH / 2) * (a.OW / 2) * 64;
      c.part = a.part + (size_t)f0 * tpf * 17 * 64;
      if (a.amax_out) c.amax_out = a.amax_out + (size_t)f0 * SFA_AMAX_WORDS;
      c.M = nf * a.OH * a.OW;
      const int nt = nf * tpf;
      const dim3 gc((unsigned)(nt < ncu ? nt : ncu));
      switch (a.stem_in) {
        case STEM_IN_NCHW3: hipLaunchKernelGGL((stem_patch_pool2_kernel<STEM_IN_NCHW3, 1>), gc, bd, 0, st, c, nt); break;
        case STEM_IN_NCHW3_FLIP:
          hipLaunchKernelGGL((stem_patch_pool2_kernel<STEM_IN_NCHW3_FLIP, 1>), gc, bd, 0, st, c, nt);
          break;
        default: hipLaunchKernelGGL((stem_patch_pool2_kernel<STEM_IN_NHWC4, 1>), gc, bd, 0, st, c, nt); break;
      }
      SFA_LAUNCH_CHECK();
    }
  } else if (a.stem_in == STEM_IN_NCHW3) {
    hipLaunchKernelGGL((stem_patch_pool_kernel<0, STEM_IN_NCHW3>), gd, bd, 0, st, a, ntiles);
  } else {
    hipLaunchKernelGGL((stem_patch_pool_kernel<0, STEM_IN_NCHW3_FLIP>), gd, bd, 0, st, a, ntiles);
  }
  SFA_LAUNCH_CHECK();
  {
    const long long n = (long long)ntiles * 15 * 16;
    hipLaunchKernelGGL(stem_pool_merge_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, frames);
  }
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

}  // namespace sfa
