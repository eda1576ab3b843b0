// FPN 1x1 convolutions (fpn_resnet.py:129-131,197-210), fp16x3, as persistent row-streaming GEMMs
// with the weight slice resident in LDS.
//
// conv_up_level{1,2,3} run commuted (model.hip): lo_f = W_a . x at the LOW resolution (no bias),
// then y = W_b . skip + b + up2x(lo_f) at the high one (the bilinear x2 align_corners upsample of
// the low-resolution product added in the epilogue: r3t_epilogue_std's res_up path).  Both are
// GEMMs with a long M (5,776 .. 369,664 rows at bs 16) and a small K x N weight slice (64 x 64 ..
// 512 x 256): HBM / latency bound, not MFMA bound (a few GFLOP over 50 .. 213 MB).  The
// per-tile kernels they ran on (conv_r3 / conv_h3: W DMA per K-tile, one 128-row tile per block,
// 2 .. 16 K-tiles) spent most of a block's life in its prologue and epilogue latencies: 1.7 .. 2.9
// TB/s.  Here:
//  * a block loads its BN-column slice of the fp16x3 weight terms ONCE into LDS (K x BN x 4 B:
//    16 .. 128 KiB; the conv_r3 swizzled fragment layout per 32-wide K-tile) and then walks row
//    tiles (128 rows: 4 waves x 2 16-row sub-tiles) of the map: grid = CUs x blocks per CU;
//  * A fragments go straight from HBM into VGPRs (a lane's 8 channels of one pixel per K-tile, as
//    conv_r3 loads them) in chunks of up to 4 K-tiles, the next chunk (the next tile's first,
//    across tile boundaries) issued before this chunk's MFMAs;
//  * the per-frame fp16x3 input scales are read once per block into LDS (rows never re-read the
//    amax shards);
//  * products, their order over K (K-tile by K-tile, hi*lo, lo*hi, hi*hi per 16x16x32 MFMA on the
//    transposed accumulators) and the epilogue are conv_r3_kernel's: the same bits as the conv_r3
//    FPN launches (R3_FPN) for the skip convs.
#pragma once

#include "conv_r3_kernel.h"

namespace sfa {

constexpr int kFpnMaxFrames = 256;

// OCC: blocks per CU the launch is built for (__launch_bounds__: 4 -> <= 128 VGPRs, 2 -> 256);
// the A chunk is 2 K-tiles at 4 blocks per CU, 4 otherwise (two chunks in flight: 2 x KC x TM x 32 B
// per lane).
template <int K, int BN, bool RU, int OCC>
struct FpnGeom {
  static constexpr int NW = 4, NT = NW * 64, WM = 32, BM = NW * WM, TM = WM / 16, TN = BN / 16;
  static constexpr int KT = K / 32;                // K-tiles
  static constexpr int KCM = OCC >= 4 ? 2 : 4;
  static constexpr int KC = KT < KCM ? KT : KCM;   // K-tiles per A chunk
  static constexpr int NCH = KT / KC;              // chunks per row tile
  static constexpr int BROW = 64, TERM_B = BN * BROW, STAGE = 2 * TERM_B, W_BYTES = KT * STAGE;
  static constexpr int LDS = W_BYTES + kFpnMaxFrames * 4 + 2 * 2 * NW * 4 + 2 * BN * 4;  // 2 amax buffers, winv / bias
  static_assert(K % 32 == 0 && KT % KC == 0 && BN % 16 == 0 && BN >= 16, "fpn geometry");
};

// r3t_epilogue_std's arithmetic (same rounding sequence: fmaf(acc * ainv, winv, b), + the
// bilinear tap value, ReLU) one 16-column block at a time, the block's residual taps loaded just
// before use (sched_barrier between blocks: hoisting every block's taps spilled at <= 128 VGPRs).
// csl: the block's columns' winv [TN * 16] and bias [TN * 16] in LDS (staged once per block: round 5,
// a global load per column block sat behind the previous block's stores)
template <int TM, int TN, int NT, bool RU>
__device__ __forceinline__ void fpn_epilogue(const ConvArgs& a, f32x4_t (&acc)[TM][TN], unsigned char* red, int mrow0,
                                             int m0, int n0, int lane, const float (&ainv)[TM], const float* csl) {
#pragma clang fp contract(off)
  const int M = a.M, c16 = lane & 15, g = lane >> 4;
  AmaxRows am(a.OH * a.OW, m0);
  int tap[TM][4];
  float wl[TM][4];
  if (RU) {
    const int H = a.OH >> 1, W = a.OW >> 1;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = min(mrow0 + mi * 16 + c16, M - 1);
      const int ow = m % a.OW, t = m / a.OW;
      const int oh = t % a.OH, b = t / a.OH;
      const float fy = a.res_sh * (float)oh, fx = a.res_sw * (float)ow;
      const int y0 = (int)fy, x0 = (int)fx;
      const int y1 = y0 + (y0 < H - 1 ? 1 : 0), x1 = x0 + (x0 < W - 1 ? 1 : 0);
      const float ly1 = fy - (float)y0, lx1 = fx - (float)x0;
      wl[mi][0] = 1.f - ly1;
      wl[mi][1] = ly1;
      wl[mi][2] = 1.f - lx1;
      wl[mi][3] = lx1;
      const int fb = b * H * W;
      tap[mi][0] = (fb + y0 * W + x0) * a.N;
      tap[mi][1] = (fb + y0 * W + x1) * a.N;
      tap[mi][2] = (fb + y1 * W + x0) * a.N;
      tap[mi][3] = (fb + y1 * W + x1) * a.N;
    }
  }
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) {
    const int n = n0 + ni * 16 + 4 * g;
    const x6_f32x4 cs = *reinterpret_cast<const x6_f32x4*>(csl + ni * 16 + 4 * g);
    const x6_f32x4 bn = *reinterpret_cast<const x6_f32x4*>(csl + TN * 16 + ni * 16 + 4 * g);
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = mrow0 + mi * 16 + c16;
      x6_f32x4 rv = {0.f, 0.f, 0.f, 0.f};
      if (RU) {
        const float* r = a.res_up + n;
        const x6_f32x4 a00 = *reinterpret_cast<const x6_f32x4*>(r + tap[mi][0]);
        const x6_f32x4 a01 = *reinterpret_cast<const x6_f32x4*>(r + tap[mi][1]);
        const x6_f32x4 a10 = *reinterpret_cast<const x6_f32x4*>(r + tap[mi][2]);
        const x6_f32x4 a11 = *reinterpret_cast<const x6_f32x4*>(r + tap[mi][3]);
        const float ly0 = wl[mi][0], ly1 = wl[mi][1], lx0 = wl[mi][2], lx1 = wl[mi][3];
#pragma unroll
        for (int v = 0; v < 4; ++v)
          rv[v] = fmaf(ly0, fmaf(lx0, a00[v], lx1 * a01[v]), ly1 * fmaf(lx0, a10[v], lx1 * a11[v]));
      }
      x6_f32x4 val;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float t = fmaf(acc[mi][ni][v] * ainv[mi], cs[v], bn[v]);
        if (RU) t += rv[v];
        if (a.relu) t = fmaxf(t, 0.f);
        val[v] = t;
      }
      if (m < M) {
        *reinterpret_cast<x6_f32x4*>(a.y + (size_t)m * a.N + n) = val;
        if (a.amax_out)
          am.add(a.amax_out, m, fmaxf(fmaxf(fabsf(val[0]), fabsf(val[1])), fmaxf(fabsf(val[2]), fabsf(val[3]))));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (a.amax_out) amax_commit_block<NT / 64>(a.amax_out, am.fb0, am.mx0, am.mx1, reinterpret_cast<float*>(red));
}

// The fp16x3 weight slice of an FPN kernel (columns n0 .. n0 + NBC - 1, KT K-tiles from column wk0 of
// the [2 terms][N][wstride] packed weights) into LDS in conv_r3's swizzled fragment layout
// [kt][term][n][16-B slot q ^ swzB(n)] (rows of 64 B, contiguous), by LDS-DMA: slot s of the region
// takes (kt, term, n, q = (s & 3) ^ swzB(n)), every piece in flight at once.  The element-wise
// load -> ds_write loop it replaces (round 5) waited one memory latency per iteration: 4 .. 32
// serialised round trips per block.  The caller waits (vmcnt(0) + barrier) before reading it.
template <int KT, int NBC, int NW>
__device__ __forceinline__ void fpn_stage_w(const ConvArgs& a, int n0, unsigned char* smem, int wave, int lane) {
  constexpr int PIECES = KT * 2 * NBC * 4 / 64;  // 64 slots of 16 B per piece
  static_assert((KT * 2 * NBC * 4) % 64 == 0, "whole pieces");
  const int wst = a.wstride ? a.wstride : a.Kpad;
  const size_t term_elems = (size_t)a.N * wst;
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.wh), (short)0,
                                                                       (int)(term_elems * 2 * 2), 0x00020000);
  auto swzB = [](int R) { return ((R >> 2) & 3) ^ ((((R & 15) + 4) >> 3) & 1); };
#pragma unroll
  for (int i = 0; i < (PIECES + NW - 1) / NW; ++i) {
    const int pc = wave + NW * i;
    if (pc >= PIECES) break;  // wave-uniform
    const int sl = pc * 64 + lane;
    const int n = (sl >> 2) % NBC, r2 = (sl >> 2) / NBC, term = r2 & 1, kt = r2 >> 1;
    const int q = (sl & 3) ^ swzB(n);
    const unsigned off = (unsigned)((term * term_elems + (size_t)(n0 + n) * wst + a.wk0 + kt * 32 + 8 * q) * 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(smem + pc * 1024), 16, off,
                                             0, 0, 0);
  }
}

template <int K, int BN, bool RU, int OCC>
__global__ void __launch_bounds__(256, OCC) fpn_gemm_kernel(const ConvArgs a, int n_mt) {
  using G = FpnGeom<K, BN, RU, OCC>;
  constexpr int NW = G::NW, NT = G::NT, WM = G::WM, BM = G::BM, TM = G::TM, TN = G::TN;
  constexpr int KC = G::KC, NCH = G::NCH, BROW = G::BROW, TERM_B = G::TERM_B, STAGE = G::STAGE;
  __shared__ __attribute__((aligned(16))) unsigned char smem[G::LDS];
  float* const FS = reinterpret_cast<float*>(smem + G::W_BYTES);  // per-frame fp16x3 scales
  // epilogue amax reduction, two buffers alternating by row tile: thread 0 reads tile t's words after
  // the commit's barrier, and a wave that runs ahead into tile t + 1 writes the other buffer (tile
  // t + 2 comes after tile t + 1's barrier, which thread 0 only reaches once it has read them)
  unsigned char* const RED = smem + G::W_BYTES + kFpnMaxFrames * 4;
  float* const CSL = reinterpret_cast<float*>(RED + 2 * 2 * NW * 4);  // [BN] winv, [BN] bias
  auto swzB = [](int R) { return ((R >> 2) & 3) ^ ((((R & 15) + 4) >> 3) & 1); };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, g = lane >> 4;
  const int bx = blockIdx.x;
  const int n0 = blockIdx.y * BN;
  const int M = a.M, P = a.OH * a.OW, nframes = (M + P - 1) / P;

  // the weight slice (columns n0 .. n0 + BN - 1, K columns from wk0) and the frame scales -> LDS
  fpn_stage_w<G::KT, BN, NW>(a, n0, smem, wave, lane);
  static_assert(2 * BN <= NT, "one winv / bias entry per thread");
  if (tid < 2 * BN) CSL[tid] = tid < BN ? a.winv[n0 + tid] : (a.bias ? a.bias[n0 + tid - BN] : 0.f);
  for (int f = tid; f < nframes; f += NT) {
    float sinv;
    FS[f] = amax_frame_scale(a.amax_in, 1, f, sinv);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.seg[0].x), (short)0,
                                                                       (int)a.seg[0].bytes, 0x00020000);
  const int bfo = c16 * BROW + ((g ^ swzB(c16)) << 4);
  const int n_my = bx < n_mt ? (n_mt - 1 - bx) / (int)gridDim.x + 1 : 0;
  const int steps = n_my * NCH;

  r3_u32x4 ra[KC][TM][2], rb[KC][TM][2];  // A chunks, ping-pong
  auto load = [&](int step, r3_u32x4 (&r)[KC][TM][2]) {
    const int t = step / NCH, c = step - t * NCH;
    const int m0 = (bx + t * (int)gridDim.x) * BM;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = m0 + wave * WM + mi * 16 + c16;
      const unsigned base = m < M ? (unsigned)(((size_t)m * K + (size_t)c * KC * 32 + 8 * g) * 4) : 0x80000000u;
#pragma unroll
      for (int kk = 0; kk < KC; ++kk) {
        const unsigned off = base == 0x80000000u ? base : base + kk * 128u;
        r[kk][mi][0] = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
        r[kk][mi][1] = __builtin_amdgcn_raw_buffer_load_b128(rsx, off + 16u, 0, 0);
      }
    }
  };
  f32x4_t acc[TM][TN];
  float as[TM], ainv[TM];
  auto process = [&](int step, r3_u32x4 (&r)[KC][TM][2]) {
    const int t = step / NCH, c = step - t * NCH;
    const int m0 = (bx + t * (int)gridDim.x) * BM;
    if (c == 0) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const int m = min(m0 + wave * WM + mi * 16 + c16, M - 1);
        as[mi] = FS[m / P];
        ainv[mi] = 1.f / as[mi];
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      f16x8_t hf[2][TM];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
        split2h_x8(__builtin_bit_cast(x6_f32x4, r[kk][mi][0]), __builtin_bit_cast(x6_f32x4, r[kk][mi][1]), as[mi],
                   hf[0][mi], hf[1][mi]);
      const unsigned char* S = smem + (c * KC + kk) * STAGE;
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const f16x8_t c0 = *reinterpret_cast<const f16x8_t*>(S + bfo + ni * 16 * BROW);
        const f16x8_t c1 = *reinterpret_cast<const f16x8_t*>(S + TERM_B + bfo + ni * 16 * BROW);
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          f32x4_t cc = acc[mi][ni];
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[1][mi], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c1, hf[0][mi], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[0][mi], cc, 0, 0, 0);
          acc[mi][ni] = cc;
        }
      }
    }
    if (c == NCH - 1) fpn_epilogue<TM, TN, NT, RU>(a, acc, RED + (t & 1) * 2 * NW * 4, m0 + wave * WM, m0, n0, lane, ainv, CSL);
  };
  // two chunks in flight: the next one's loads issued before this one's MFMAs; one copy of the
  // body (rb is moved into ra, which the next iteration's MFMAs would wait for anyway)
  if (steps > 0) load(0, ra);
  for (int s = 0; s < steps; ++s) {
    if (s + 1 < steps) load(s + 1, rb);
    process(s, ra);
#pragma unroll
    for (int kk = 0; kk < KC; ++kk)
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        ra[kk][mi][0] = rb[kk][mi][0];
        ra[kk][mi][1] = rb[kk][mi][1];
      }
  }
}

// One FPN 1x1 conv (one segment, 1x1 / stride 1, K = its channel count, weight slice by
// wstride / wk0, optional half-resolution residual res_up); SFA_E_UNSUPPORTED for other shapes.
template <int K, int BN, bool RU, int OCC>
inline int launch_fpn_gemm_cfg(const ConvArgs& a, hipStream_t st) {
  using G = FpnGeom<K, BN, RU, OCC>;
  static_assert(OCC * G::LDS <= 160 * 1024, "blocks per CU vs LDS");
  const ConvSeg& g = a.seg[0];
  if (a.nseg != 1 || g.KH != 1 || g.KW != 1 || g.stride != 1 || g.pad != 0 || g.C != K || a.Kpad != K ||
      a.N % BN != 0 || !a.wh || !a.winv || a.res || a.ksplit > 1 || a.OH != g.H || a.OW != g.W ||
      (a.res_up != nullptr) != RU || (a.wstride && (a.wstride < a.wk0 + K || a.wk0 % 8 != 0))) {
    set_error("fpn_gemm: not a 1x1 conv with C = %d (N=%d)", K, a.N);
    return SFA_E_UNSUPPORTED;
  }
  const int P = a.OH * a.OW;
  if (2ull * a.N * (a.wstride ? a.wstride : a.Kpad) * 2ull >= (1ull << 31)) {
    set_error("fpn_gemm: weights >= 2 GiB");
    return SFA_E_UNSUPPORTED;
  }
  const int frames = (a.M + P - 1) / P;
  if (frames > kFpnMaxFrames) {
    // the per-frame scale table holds kFpnMaxFrames frames: launch frame chunks of that size. A row's
    // products, K order and epilogue do not depend on the block that computes it, so every frame gets
    // the bits it gets in a smaller batch (batch invariance).
    if (a.M != frames * P) {
      set_error("fpn_gemm: M=%d is not a whole number of %d-pixel frames", a.M, P);
      return SFA_E_INVALID;
    }
    const size_t half = (size_t)(a.OH / 2) * (a.OW / 2) * a.N;  // res_up floats per frame
    for (int f0 = 0; f0 < frames; f0 += kFpnMaxFrames) {
      const int nf = frames - f0 < kFpnMaxFrames ? frames - f0 : kFpnMaxFrames;
      ConvArgs c = a;
      c.M = nf * P;
      c.seg[0].x = a.seg[0].x + (size_t)f0 * P * K;
      c.seg[0].bytes = (unsigned)((size_t)c.M * K * 4);
      c.y = a.y + (size_t)f0 * P * a.N;
      if (a.amax_in[0]) c.amax_in[0] = a.amax_in[0] + (size_t)f0 * SFA_AMAX_WORDS;
      if (a.amax_out) c.amax_out = a.amax_out + (size_t)f0 * SFA_AMAX_WORDS;
      if (RU) c.res_up = a.res_up + (size_t)f0 * half;
      const int rc = launch_fpn_gemm_cfg<K, BN, RU, OCC>(c, st);
      if (rc != SFA_OK) return rc;
    }
    return SFA_OK;
  }
  const int ncu = cu_count(st);
  const int n_mt = ceil_div(a.M, G::BM), n_nt = a.N / BN;
  int gx = (ncu * OCC + n_nt - 1) / n_nt;  // blocks per column tile
  if (gx > n_mt) gx = n_mt;
  if (gx < 1) return SFA_OK;
  hipLaunchKernelGGL((fpn_gemm_kernel<K, BN, RU, OCC>), dim3((unsigned)gx, (unsigned)n_nt), dim3(G::NT), 0, st, a,
                     n_mt);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}


// FPN skip convs (up_level = W_b . skip + b + up2x(W_a . x), the upsampled residual added in the
// epilogue) on full output rows (round 4).  The per-tile kernels (conv_r3 R3_FPN, fpn_gemm above)
// gather the epilogue's four bilinear taps from L2 just before use — 16 float4 loads per lane per
// 32-row tile, their latency exposed (PMC: waves waiting 70 % of their cycles on the 152-wide level,
// 3.1 TB/s).  Here a block walks the rows of one frame segment for one 64-channel column tile; the
// half-resolution source rows the taps need live in an LDS ring of 3 rows (each loaded ONCE per
// segment by LDS-DMA, one row ahead: output row y needs source rows y0(y), y0(y) + 1 and y0 advances
// by at most one per output row), the weight slice and the channels' scales / biases in LDS, and the
// next row's A fragments are issued right after this row's split, before its MFMAs.  Products, K
// order, split and the epilogue's rounding sequence are conv_r3_kernel's (R3_FPN): the same bits.
namespace fpn_row {
constexpr int NT = 256, NW = 4, NB = 64, TNB = NB / 16;  // 64 output channels per block
constexpr int BROW = 64, TERM_B = NB * BROW, STAGE = 2 * TERM_B;
// RB row blocks of 16 pixels per output row (W <= 16 RB); source rows of W / 2 <= 8 RB pixels
__host__ __device__ constexpr int slot_bytes(int RB) { return 8 * RB * NB * 4; }
__host__ __device__ constexpr int lds_bytes(int K, int RB) { return (K / 32) * STAGE + 3 * slot_bytes(RB) + 2 * NB * 4 + NW * 4; }
}  // namespace fpn_row

template <int K, int RB, int OCC>
__global__ void __launch_bounds__(256, OCC) fpn_row_kernel(const ConvArgs a, int segs) {
#pragma clang fp contract(off)
  using namespace fpn_row;
  constexpr int KT = K / 32, W_BYTES = KT * STAGE;
  constexpr int RBW = (RB + NW - 1) / NW;  // row blocks per wave (wave w: w, w + NW, ..)
  constexpr int SLOT = slot_bytes(RB);
  static_assert(OCC * lds_bytes(K, RB) <= 160 * 1024, "blocks per CU vs LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[lds_bytes(K, RB)];
  unsigned char* const ring = smem + W_BYTES;
  float* const CSB = reinterpret_cast<float*>(smem + W_BYTES + 3 * SLOT);  // [NB] winv, [NB] bias
  float* const red = CSB + 2 * NB;
  auto swzB = [](int R) { return ((R >> 2) & 3) ^ ((((R & 15) + 4) >> 3) & 1); };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, g = lane >> 4;
  const int H = a.OH, W = a.OW, Hh = H >> 1, Wh = W >> 1, N = a.N;
  const int nct = N / NB;
  // the nct column tiles of one segment on consecutive logical ids, i.e. on one XCD: they read the same
  // A rows, which its L2 then serves once (round 6: blockIdx order put them on nct XCDs, nct x the reads)
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int ct = lb % nct, rest = lb / nct;
  const int b = rest / segs, sk = rest - b * segs;
  const int n0 = ct * NB;
  const int y0 = sk * H / segs, y1 = (sk + 1) * H / segs;
  if (y1 <= y0) return;  // uniform per block

  // the weight slice (columns n0 .., K columns from wk0) in conv_r3's swizzled fragment layout
  fpn_stage_w<KT, NB, NW>(a, n0, smem, wave, lane);
  if (tid < NB) {  // both loads in flight before either store (NB <= NT)
    const float wv = a.winv[n0 + tid], bv = a.bias ? a.bias[n0 + tid] : 0.f;
    CSB[tid] = wv;
    CSB[NB + tid] = bv;
  }
  float ainv;
  const float as = amax_frame_scale(a.amax_in, 1, b, ainv);
  ainv = 1.f / as;  // as conv_r3 forms it

  // source rows (half resolution): the block's NB channels of each pixel, by LDS-DMA (16 B per lane,
  // LDS in item order = [pixel][NB channels])
  const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.res_up), (short)0, (int)((size_t)(a.M / (H * W)) * Hh * Wh * N * 4), 0x00020000);
  const int items = Wh * (NB / 4);
  auto dma_src = [&](int sy) {
    unsigned char* dst = ring + (sy % 3) * SLOT;
    const size_t rbase = ((size_t)(b * Hh + sy) * Wh) * N + n0;  // floats
    for (int piece = wave; piece * 64 < items; piece += NW) {
      const int it = piece * 64 + lane;
      const unsigned off = it < items ? (unsigned)((rbase + (size_t)(it / (NB / 4)) * N + 4 * (it % (NB / 4))) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsr, (__attribute__((address_space(3))) void*)(dst + piece * 1024), 16,
                                               off, 0, 0, 0);
    }
  };
  auto srow0 = [&](int y) { return (int)(a.res_sh * (float)y); };

  // A: lane (c16, g) of row block rb -> pixel 16 rb + c16, channels 32 kt + 8 g .. + 7
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.seg[0].x), (short)0,
                                                                       (int)a.seg[0].bytes, 0x00020000);
  r3_u32x4 ra[RBW][KT][2];
  auto load_a = [&](int y) {
#pragma unroll
    for (int i = 0; i < RBW; ++i) {
      const int x = 16 * (wave + NW * i) + c16;
      const bool ok = wave + NW * i < RB && x < W;
      const unsigned base = ok ? (unsigned)((((size_t)(b * H + y) * W + x) * K + 8 * g) * 4) : 0x80000000u;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const unsigned off = ok ? base + kt * 128u : base;
        ra[i][kt][0] = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
        ra[i][kt][1] = __builtin_amdgcn_raw_buffer_load_b128(rsx, off + 16u, 0, 0);
      }
    }
  };

  // prologue: source rows of the first output row, its A fragments
  int hi_row = min(srow0(y0) + 1, Hh - 1);  // highest source row in the ring
  for (int sy = srow0(y0); sy <= hi_row; ++sy) dma_src(sy);
  load_a(y0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int bfo = c16 * BROW + ((g ^ swzB(c16)) << 4);
  float tmx = 0.f;
  for (int y = y0; y < y1; ++y) {
    // the source row the next output row may need beyond the ring's top (its slot held a row <= y0(y) - 1)
    const int want = min(srow0(y) + 2, Hh - 1);
    if (y + 1 < y1 && want > hi_row) {
      dma_src(want);
      hi_row = want;
    }
    // this row's A split into fp16 terms first, so the next row's loads go out before the MFMAs
    f16x8_t hf[RBW][KT][2];
#pragma unroll
    for (int i = 0; i < RBW; ++i)
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
        split2h_x8(__builtin_bit_cast(x6_f32x4, ra[i][kt][0]), __builtin_bit_cast(x6_f32x4, ra[i][kt][1]), as,
                   hf[i][kt][0], hf[i][kt][1]);
    if (y + 1 < y1) load_a(y + 1);  // the next row's A flies during this row's MFMAs and epilogue
    f32x4_t acc[RBW][TNB];
#pragma unroll
    for (int i = 0; i < RBW; ++i) {
#pragma unroll
      for (int ni = 0; ni < TNB; ++ni) acc[i][ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const unsigned char* S = smem + kt * STAGE;
#pragma unroll
        for (int ni = 0; ni < TNB; ++ni) {
          const f16x8_t c0 = *reinterpret_cast<const f16x8_t*>(S + bfo + ni * 16 * BROW);
          const f16x8_t c1 = *reinterpret_cast<const f16x8_t*>(S + TERM_B + bfo + ni * 16 * BROW);
          f32x4_t cc = acc[i][ni];
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[i][kt][1], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c1, hf[i][kt][0], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[i][kt][0], cc, 0, 0, 0);
          acc[i][ni] = cc;
        }
      }
    }
    // epilogue (r3t_epilogue_std with the upsampled residual): taps from the ring
    const float fy = a.res_sh * (float)y;
    const int sy0 = (int)fy, sy1 = sy0 + (sy0 < Hh - 1 ? 1 : 0);
    const float ly1 = fy - (float)sy0, ly0 = 1.f - ly1;
    const unsigned char* R0 = ring + (sy0 % 3) * SLOT;
    const unsigned char* R1 = ring + (sy1 % 3) * SLOT;
#pragma unroll
    for (int i = 0; i < RBW; ++i) {
      const int x = 16 * (wave + NW * i) + c16;
      if (wave + NW * i >= RB) continue;  // wave-uniform
      const float fx = a.res_sw * (float)x;
      const int sx0 = (int)fx, sx1 = sx0 + (sx0 < Wh - 1 ? 1 : 0);
      const float lx1 = fx - (float)sx0, lx0 = 1.f - lx1;
      const bool in = x < W;
      const int o0 = (in ? sx0 : 0) * NB * 4, o1 = (in ? sx1 : 0) * NB * 4;
#pragma unroll
      for (int ni = 0; ni < TNB; ++ni) {
        const int n = ni * 16 + 4 * g;
        const x6_f32x4 a00 = *reinterpret_cast<const x6_f32x4*>(R0 + o0 + n * 4);
        const x6_f32x4 a01 = *reinterpret_cast<const x6_f32x4*>(R0 + o1 + n * 4);
        const x6_f32x4 a10 = *reinterpret_cast<const x6_f32x4*>(R1 + o0 + n * 4);
        const x6_f32x4 a11 = *reinterpret_cast<const x6_f32x4*>(R1 + o1 + n * 4);
        const x6_f32x4 cs = *reinterpret_cast<const x6_f32x4*>(CSB + n);
        const x6_f32x4 bn = *reinterpret_cast<const x6_f32x4*>(CSB + NB + n);
        x6_f32x4 val;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float rv = fmaf(ly0, fmaf(lx0, a00[v], lx1 * a01[v]), ly1 * fmaf(lx0, a10[v], lx1 * a11[v]));
          float t = fmaf(acc[i][ni][v] * ainv, cs[v], bn[v]);
          t += rv;
          if (a.relu) t = fmaxf(t, 0.f);
          val[v] = t;
        }
        if (in) {
          *reinterpret_cast<x6_f32x4*>(a.y + ((size_t)(b * H + y) * W + x) * N + n0 + n) = val;
          tmx = fmaxf(tmx, fmaxf(fmaxf(fabsf(val[0]), fabsf(val[1])), fmaxf(fabsf(val[2]), fabsf(val[3]))));
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next row's A and this wave's DMA pieces
    __syncthreads();  // the ring slot written above is visible; every wave is done with this row's taps
  }
  if (a.amax_out) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) tmx = fmaxf(tmx, __shfl_xor(tmx, o, 64));
    if (lane == 0) red[wave] = tmx;
    __syncthreads();
    if (tid == 0) {
      float m = red[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) m = fmaxf(m, red[w]);
      if (m > 0.f) amax_atomic(a.amax_out, b, m);
    }
  }
}

// An FPN skip conv (1x1, K = C, N a multiple of 64, the upsampled residual) on full output rows: the
// three KFPN levels' shapes (K 64 / 128 / 256 at widths <= 160 / 80 / 48, even output dims);
// SFA_E_UNSUPPORTED otherwise.
template <int K, int RB, int OCC>
inline int launch_fpn_row_cfg(const ConvArgs& a, hipStream_t st) {
  using namespace fpn_row;
  const ConvSeg& g = a.seg[0];
  if (a.nseg != 1 || g.KH != 1 || g.KW != 1 || g.stride != 1 || g.pad != 0 || g.C != K || a.Kpad != K ||
      a.N % NB != 0 || !a.wh || !a.winv || a.res || !a.res_up || a.ksplit > 1 || a.OH != g.H || a.OW != g.W ||
      a.OH % 2 || a.OW % 2 || a.OW > 16 * RB || (a.wstride && (a.wstride < a.wk0 + K || a.wk0 % 8 != 0)))
    return SFA_E_UNSUPPORTED;
  const int frames = a.M / (a.OH * a.OW);
  if (frames <= 0) return SFA_OK;
  if ((size_t)frames * (a.OH / 2) * (a.OW / 2) * a.N * 4 >= (1ull << 31)) return SFA_E_UNSUPPORTED;
  const int ncu = cu_count(st);
  const int nct = a.N / NB;
  int segs = (OCC * ncu + frames * nct - 1) / (frames * nct);  // about OCC blocks per CU
  segs = segs < 1 ? 1 : (segs > a.OH ? a.OH : segs);
  hipLaunchKernelGGL((fpn_row_kernel<K, RB, OCC>), dim3((unsigned)(frames * segs * nct)), dim3(NT), 0, st, a, segs);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

// FPN skip convs of the narrow levels (round 5): fpn_row_kernel walks one output
// row per step, which at 76 / 38 pixels is 2.4 - 4.75 row blocks of 16 for 4 waves, a barrier and an
// exposed load latency per row (profiles/r04m_*: slower than conv_r3 there).  Here a block walks its
// frame segment as a FLAT pixel range in steps of 16 NW pixels (one 16-pixel block per wave, rows
// crossed freely): every wave has work each step and a step covers 1.7 - 3.4 output rows.  The
// half-resolution source rows of the residual taps live in an LDS ring of NSLOT rows (row r in slot
// r % NSLOT), the rows the next step needs loaded by LDS-DMA during this one; each lane finds its own
// pixel's (y, x), tap rows and weights.  Weight slice, scales / biases in LDS and the next step's A
// fragments issued before this step's MFMAs, as fpn_row_kernel; products, K order, split and the
// epilogue's rounding sequence are conv_r3_kernel's (R3_FPN): the same bits.
namespace fpn_seg {
constexpr int NW = 8, NT = 64 * NW, NB = 64, TNB = NB / 16, P = 16 * NW;  // pixels per step
constexpr int BROW = 64, TERM_B = NB * BROW, STAGE = 2 * TERM_B;
constexpr int WHMAX = 40, NSLOT = 8, SLOT = WHMAX * NB * 4;  // source rows of <= 40 pixels
__host__ __device__ constexpr int lds_bytes(int K) { return (K / 32) * STAGE + NSLOT * SLOT + 2 * NB * 4 + NW * 4; }
// the source rows one step (pixels [p, p + P) of rows y0 .. y1 - 1) reads: [lo, hi]
__host__ __device__ inline void step_rows(int p, int pend, int W, int Hh, float sh, int& lo, int& hi) {
  const int ya = p / W, yb = (min(p + P, pend) - 1) / W;
  lo = (int)(sh * (float)ya);
  hi = min((int)(sh * (float)yb) + 1, Hh - 1);
}
}  // namespace fpn_seg

template <int K, int OCC>
__global__ void __launch_bounds__(fpn_seg::NT, OCC) fpn_seg_kernel(const ConvArgs a, int segs) {
#pragma clang fp contract(off)
  using namespace fpn_seg;
  constexpr int KT = K / 32, W_BYTES = KT * STAGE;
  __shared__ __attribute__((aligned(16))) unsigned char smem[lds_bytes(K)];
  unsigned char* const ring = smem + W_BYTES;
  float* const CSB = reinterpret_cast<float*>(smem + W_BYTES + NSLOT * SLOT);  // [NB] winv, [NB] bias
  float* const red = CSB + 2 * NB;
  auto swzB = [](int R) { return ((R >> 2) & 3) ^ ((((R & 15) + 4) >> 3) & 1); };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, g = lane >> 4;
  const int H = a.OH, W = a.OW, Hh = H >> 1, Wh = W >> 1, N = a.N;
  const int nct = N / NB;
  // the nct column tiles of one segment on consecutive logical ids, i.e. on one XCD: they read the same
  // A rows, which its L2 then serves once (round 6: blockIdx order put them on nct XCDs, nct x the reads)
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int ct = lb % nct, rest = lb / nct;
  const int b = rest / segs, sk = rest - b * segs;
  const int n0 = ct * NB;
  const int pbeg = (sk * H / segs) * W, pend = ((sk + 1) * H / segs) * W;  // the segment's pixels
  if (pend <= pbeg) return;  // uniform per block

  // the weight slice (columns n0 .., K columns from wk0) in conv_r3's swizzled fragment layout
  fpn_stage_w<KT, NB, NW>(a, n0, smem, wave, lane);
  if (tid < NB) {  // both loads in flight before either store (NB <= NT)
    const float wv = a.winv[n0 + tid], bv = a.bias ? a.bias[n0 + tid] : 0.f;
    CSB[tid] = wv;
    CSB[NB + tid] = bv;
  }
  float ainv;
  const float as = amax_frame_scale(a.amax_in, 1, b, ainv);
  ainv = 1.f / as;  // as conv_r3 forms it

  // source rows (half resolution): the block's NB channels of each pixel by LDS-DMA (16 B per lane,
  // LDS in item order = [pixel][NB channels]); the pieces of consecutive rows spread over the waves
  const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.res_up), (short)0, (int)((size_t)(a.M / (H * W)) * Hh * Wh * N * 4), 0x00020000);
  const int items = Wh * (NB / 4), npc = (items + 63) >> 6;
  auto dma_rows = [&](int r0, int r1) {  // rows r0 .. r1
    for (int u = wave; u < (r1 - r0 + 1) * npc; u += NW) {
      const int sy = r0 + u / npc, piece = u - (u / npc) * npc;
      const int it = piece * 64 + lane;
      const size_t rbase = ((size_t)(b * Hh + sy) * Wh) * N + n0;  // floats
      const unsigned off = it < items ? (unsigned)((rbase + (size_t)(it / (NB / 4)) * N + 4 * (it % (NB / 4))) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsr, (__attribute__((address_space(3))) void*)(ring + (sy % NSLOT) * SLOT + piece * 1024), 16, off, 0, 0, 0);
    }
  };

  // A: lane (c16, g) -> pixel p + 16 wave + c16 of the frame, channels 32 kt + 8 g .. + 7
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.seg[0].x), (short)0,
                                                                       (int)a.seg[0].bytes, 0x00020000);
  const size_t fpix = (size_t)b * H * W;  // the frame's first pixel
  r3_u32x4 ra[KT][2];
  auto load_a = [&](int p) {
    const int q = p + 16 * wave + c16;
    const bool ok = q < pend;
    const unsigned base = ok ? (unsigned)(((fpix + q) * K + 8 * g) * 4) : 0x80000000u;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const unsigned off = ok ? base + kt * 128u : base;
      ra[kt][0] = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
      ra[kt][1] = __builtin_amdgcn_raw_buffer_load_b128(rsx, off + 16u, 0, 0);
    }
  };

  // prologue: the first step's source rows and A fragments
  int lo, hi;
  step_rows(pbeg, pend, W, Hh, a.res_sh, lo, hi);
  dma_rows(lo, hi);
  load_a(pbeg);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int bfo = c16 * BROW + ((g ^ swzB(c16)) << 4);
  float tmx = 0.f;
  for (int p = pbeg; p < pend; p += P) {
    const bool more = p + P < pend;
    // the rows the next step needs beyond this one's (slots of rows below this step's lowest: free)
    if (more) {
      int lo2, hi2;
      step_rows(p + P, pend, W, Hh, a.res_sh, lo2, hi2);
      if (hi2 > hi) dma_rows(max(hi + 1, lo2), hi2);
      hi = hi2;
    }
    // this step's A split into fp16 terms first, so the next step's loads go out before the MFMAs
    f16x8_t hf[KT][2];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
      split2h_x8(__builtin_bit_cast(x6_f32x4, ra[kt][0]), __builtin_bit_cast(x6_f32x4, ra[kt][1]), as, hf[kt][0],
                 hf[kt][1]);
    if (more) load_a(p + P);
    f32x4_t acc[TNB];
#pragma unroll
    for (int ni = 0; ni < TNB; ++ni) acc[ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const unsigned char* S = smem + kt * STAGE;
#pragma unroll
      for (int ni = 0; ni < TNB; ++ni) {
        const f16x8_t c0 = *reinterpret_cast<const f16x8_t*>(S + bfo + ni * 16 * BROW);
        const f16x8_t c1 = *reinterpret_cast<const f16x8_t*>(S + TERM_B + bfo + ni * 16 * BROW);
        f32x4_t cc = acc[ni];
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[kt][1], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c1, hf[kt][0], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[kt][0], cc, 0, 0, 0);
        acc[ni] = cc;
      }
    }
    // epilogue (r3t_epilogue_std with the upsampled residual): this lane's pixel, taps from the ring
    const int q = p + 16 * wave + c16;
    const bool in = q < pend;
    const int y = in ? q / W : 0, x = in ? q - y * W : 0;
    const float fy = a.res_sh * (float)y;
    const int sy0 = (int)fy, sy1 = sy0 + (sy0 < Hh - 1 ? 1 : 0);
    const float ly1 = fy - (float)sy0, ly0 = 1.f - ly1;
    const float fx = a.res_sw * (float)x;
    const int sx0 = (int)fx, sx1 = sx0 + (sx0 < Wh - 1 ? 1 : 0);
    const float lx1 = fx - (float)sx0, lx0 = 1.f - lx1;
    const unsigned char* R0 = ring + (sy0 % NSLOT) * SLOT;
    const unsigned char* R1 = ring + (sy1 % NSLOT) * SLOT;
    const int o0 = sx0 * NB * 4, o1 = sx1 * NB * 4;
#pragma unroll
    for (int ni = 0; ni < TNB; ++ni) {
      const int n = ni * 16 + 4 * g;
      const x6_f32x4 a00 = *reinterpret_cast<const x6_f32x4*>(R0 + o0 + n * 4);
      const x6_f32x4 a01 = *reinterpret_cast<const x6_f32x4*>(R0 + o1 + n * 4);
      const x6_f32x4 a10 = *reinterpret_cast<const x6_f32x4*>(R1 + o0 + n * 4);
      const x6_f32x4 a11 = *reinterpret_cast<const x6_f32x4*>(R1 + o1 + n * 4);
      const x6_f32x4 cs = *reinterpret_cast<const x6_f32x4*>(CSB + n);
      const x6_f32x4 bn = *reinterpret_cast<const x6_f32x4*>(CSB + NB + n);
      x6_f32x4 val;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float rv = fmaf(ly0, fmaf(lx0, a00[v], lx1 * a01[v]), ly1 * fmaf(lx0, a10[v], lx1 * a11[v]));
        float t = fmaf(acc[ni][v] * ainv, cs[v], bn[v]);
        t += rv;
        if (a.relu) t = fmaxf(t, 0.f);
        val[v] = t;
      }
      if (in) {
        *reinterpret_cast<x6_f32x4*>(a.y + (fpix + q) * N + n0 + n) = val;
        tmx = fmaxf(tmx, fmaxf(fmaxf(fabsf(val[0]), fabsf(val[1])), fmaxf(fabsf(val[2]), fabsf(val[3]))));
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next step's A and this wave's DMA pieces
    __syncthreads();  // the ring rows written above are visible; every wave is done with this step's taps
  }
  if (a.amax_out) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) tmx = fmaxf(tmx, __shfl_xor(tmx, o, 64));
    if (lane == 0) red[wave] = tmx;
    __syncthreads();
    if (tid == 0) {
      float m = red[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) m = fmaxf(m, red[w]);
      if (m > 0.f) amax_atomic(a.amax_out, b, m);
    }
  }
}

// An FPN skip conv on flat pixel steps: K = C 128 / 256, N a multiple of 64, even output dims, source
// rows of <= WHMAX pixels, and every two consecutive steps' source rows within the ring (checked here
// over the launch's segments); SFA_E_UNSUPPORTED otherwise.
template <int K, int OCC>
inline int launch_fpn_seg_cfg(const ConvArgs& a, hipStream_t st) {
  using namespace fpn_seg;
  static_assert(OCC * lds_bytes(K) <= 160 * 1024, "blocks per CU vs LDS");
  const ConvSeg& g = a.seg[0];
  if (a.nseg != 1 || g.KH != 1 || g.KW != 1 || g.stride != 1 || g.pad != 0 || g.C != K || a.Kpad != K ||
      a.N % NB != 0 || !a.wh || !a.winv || a.res || !a.res_up || a.ksplit > 1 || a.OH != g.H || a.OW != g.W ||
      a.OH % 2 || a.OW % 2 || a.OW / 2 > WHMAX || (a.wstride && (a.wstride < a.wk0 + K || a.wk0 % 8 != 0)))
    return SFA_E_UNSUPPORTED;
  const int frames = a.M / (a.OH * a.OW);
  if (frames <= 0) return SFA_OK;
  if ((size_t)frames * a.OH * a.OW * K * 4 >= (1ull << 31) ||
      (size_t)frames * (a.OH / 2) * (a.OW / 2) * a.N * 4 >= (1ull << 31))
    return SFA_E_UNSUPPORTED;
  const int ncu = cu_count(st);
  const int nct = a.N / NB;
  int segs = (OCC * ncu + frames * nct - 1) / (frames * nct);  // about OCC blocks per CU
  segs = segs < 1 ? 1 : (segs > a.OH ? a.OH : segs);
  // the ring holds every two consecutive steps' source rows (the same for every frame)
  const int H = a.OH, W = a.OW, Hh = H / 2;
  for (int sk = 0; sk < segs; ++sk) {
    const int pb = (sk * H / segs) * W, pe = ((sk + 1) * H / segs) * W;
    for (int p = pb; p < pe; p += P) {
      int lo, hi, lo2 = 0, hi2 = 0;
      step_rows(p, pe, W, Hh, a.res_sh, lo, hi);
      if (p + P < pe) step_rows(p + P, pe, W, Hh, a.res_sh, lo2, hi2);
      if (max(hi, hi2) - lo + 1 > NSLOT || (p + P < pe && lo2 < lo)) return SFA_E_UNSUPPORTED;
    }
  }
  hipLaunchKernelGGL((fpn_seg_kernel<K, OCC>), dim3((unsigned)(frames * segs * nct)), dim3(NT), 0, st, a, segs);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

// the skip conv of each KFPN level by its input channel count (the 608-input widths 152 / 76 / 38 and
// the test sizes' 48 / 24 / 12 .. 40 / 20 / 10)
inline int launch_fpn_row(const ConvArgs& a, hipStream_t st) {
  const int C = a.seg[0].C, W = a.OW;
  if (C == 64) return W > 80 ? launch_fpn_row_cfg<64, 10, 2>(a, st) : launch_fpn_row_cfg<64, 5, 2>(a, st);
  if (C == 128) return W > 48 ? launch_fpn_row_cfg<128, 5, 1>(a, st) : launch_fpn_row_cfg<128, 3, 2>(a, st);
  if (C == 256) return launch_fpn_row_cfg<256, 3, 1>(a, st);
  return SFA_E_UNSUPPORTED;
}

}  // namespace sfa
