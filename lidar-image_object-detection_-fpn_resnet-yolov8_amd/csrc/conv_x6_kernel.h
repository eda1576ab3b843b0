// Implicit-GEMM convolution on bf16 MFMA with an f32-accurate 3-way operand split
// ("bf16x6") for gfx950 (CDNA4).
//
// Same GEMM view as conv_kernel.h (C[M][N] = A[M][K] * W[N][K]^T over NHWC, two
// K-segments, fused epilogues), but every f32 operand x is carried as three bf16
// terms x = x0 + x1 + x2 (x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1);
// each difference is exact in f32, so the three terms hold all 24 significand bits)
// and each product is formed from the six terms that are not below f32 rounding:
//   a*w ~= a0w0 + a0w1 + a1w0 + a1w1 + a0w2 + a2w0     (dropped: O(2^-24) a*w)
// on v_mfma_f32_32x32x16_bf16 (bf16 x bf16 products are exact, f32 accumulation).
// Six bf16 MFMAs cost 6/16 of the f32 MFMA time for the same MACs: the f32-input
// MFMA runs at 1/16 of the bf16 rate on gfx950 (no xf32 / TF32 form exists).
// Measured on the KFPN e2e frame (torch emulation, /oracle fixtures): max rel. logit
// error 2.9e-6 — below the f32 MFMA path's own 7.3e-6 vs the reference.
//
// Operand layout of v_mfma_f32_32x32x16_bf16: lane l = (r = l & 31, h = l >> 5)
// feeds row/column r with k = 8h .. 8h+7 of the 16-deep k-step: one 16-B chunk of
// its row.  LDS tiles are [rows][BK] bf16 per term; 16-B chunk c of row R is stored
// at chunk c ^ swz(R) so the ds_read_b128 lane groups hit 16 distinct bank groups:
// swz = (R >> 3) & 1 for 32-B rows (BK = 16), (R >> 2) & 3 for 64-B rows (BK = 32).
// A (activations) is gathered in f32 with buffer loads (out-of-window taps -> 0, as
// conv_kernel.h) and split while it is written to LDS; W was split on the host.
#pragma once

#include <type_traits>

#include "conv.h"

namespace sfa {

typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float x6_f32x16 __attribute__((ext_vector_type(16)));
typedef float x6_f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned x6_u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(const x6_f32x4 v, bf16x4_t& t0, bf16x4_t& t1, bf16x4_t& t2) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const __bf16 a = (__bf16)v[i];
    const float r = v[i] - (float)a;
    const __bf16 b = (__bf16)r;
    t0[i] = a;
    t1[i] = b;
    t2[i] = (__bf16)(r - (float)b);
  }
}

// fp16x3: x * s = hi + lo with hi = fp16(x * s), lo = fp16(x * s - hi) (the difference is
// exact in f32): 22 significand bits; s is a power of two, so x * s is exact.
__device__ __forceinline__ void split2h(const x6_f32x4 v, float s, f16x4_t& t0, f16x4_t& t1) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x = v[i] * s;
    const _Float16 hi = (_Float16)x;
    t0[i] = hi;
    t1[i] = (_Float16)(x - (float)hi);
  }
}

// The same split in 2 VALU per value (hipcc mixes v_pk_mul / v_cvt_pk / v_cvt_f32_f16 / v_pk_fma
// in and needs ~3.5): per pair, hi by v_fma_mixlo / mixhi (x s rounded once to fp16; x s is
// exact), lo by the same with the fp16 hi as a negated third source (x s - hi is exact in f32,
// rounded once). Bit-identical to split2h.
__device__ __forceinline__ void split2h_pair(float x0, float x1, float s, unsigned& hi2, unsigned& lo2) {
  asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(hi2), "=&v"(lo2)
      : "v"(x0), "v"(x1), "v"(s));
}
// 8 f32 values (two quads) -> the fp16 hi / lo fragments (f16x8) of an MFMA operand
__device__ __forceinline__ void split2h_x8(const x6_f32x4 q0, const x6_f32x4 q1, float s, f16x8_t& hi, f16x8_t& lo) {
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  unsigned h0, h1, h2, h3, l0, l1, l2, l3;
  split2h_pair(q0[0], q0[1], s, h0, l0);
  split2h_pair(q0[2], q0[3], s, h1, l1);
  split2h_pair(q1[0], q1[1], s, h2, l2);
  split2h_pair(q1[2], q1[3], s, h3, l3);
  hi = __builtin_bit_cast(f16x8_t, u32x4_t{h0, h1, h2, h3});
  lo = __builtin_bit_cast(f16x8_t, u32x4_t{l0, l1, l2, l3});
}

// Shared epilogue of the bf16x6 kernels (the accumulator layout of every 32x32 MFMA:
// lane (r, h), register v -> row (v & 3) + 8 (v >> 2) + 4h, column r).
// PREC 1 (fp16x3): the accumulator of row R holds sum (x s_R)(w 2^e[n]); it is scaled
// back by 1/s_R (ainv[mi] of the lane holding row R as its A row) and winv[n], both
// powers of two, before the bias.  amax_out: the output's per-frame max |y| (conv.h).
template <int BM, int BN, int WM, int WN, int TM, int TN, int NT, int EPI, int PREC = 0, bool RES_UP = true>
__device__ __forceinline__ void x6_epilogue(const ConvArgs& a, x6_f32x16 (&acc)[TM][TN],
                                            unsigned char* smem, int m0, int n0, int nt, int wm,
                                            int wn, int tid, const float (&ainv)[TM]) {
  constexpr int HCH = BM < 128 ? BM : 128;
  const int M = a.M, lane = tid & 63, r = lane & 31, h = lane >> 5;
  // row scales in accumulator order (lane (r, h), register v -> tile row (v&3)+8(v>>2)+4h)
  float rinv[TM][16];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int v = 0; v < 16; ++v)
      rinv[mi][v] = PREC ? __shfl(ainv[mi], (v & 3) + 8 * (v >> 2) + 4 * h, 64) : 1.f;
  if constexpr (EPI == EPI_STD) {
    AmaxRows am(a.OH * a.OW, m0);
    // residual tile loaded up front (one latency for all of it, not one per element)
    float rv[TM][TN][16];
    if (a.res) {
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int m = min(m0 + wm * WM + mi * 32 + (v & 3) + 8 * (v >> 2) + 4 * h, M - 1);
            rv[mi][ni][v] = a.res[(size_t)m * a.N + n0 + wn * WN + ni * 32 + r];
          }
    }
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      // the upsampled residual (4 taps per value) is sampled per column block, not hoisted for the
      // whole tile: that would hold 4 x TM x TN x 16 loads in registers and spill
      if (RES_UP && a.res_up) {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int m = min(m0 + wm * WM + mi * 32 + (v & 3) + 8 * (v >> 2) + 4 * h, M - 1);
            rv[mi][ni][v] = res_up_sample(a, m, n0 + wn * WN + ni * 32 + r);
          }
      }
      const int n = n0 + wn * WN + ni * 32 + r;
      const float bn = a.bias ? a.bias[n] : 0.f;
      const float cs = PREC ? a.winv[n] : 1.f;
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int m = m0 + wm * WM + mi * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          if (m < M) {
            float val = (PREC ? acc[mi][ni][v] * rinv[mi][v] * cs : acc[mi][ni][v]) + bn;
            if (a.res || (RES_UP && a.res_up)) val += rv[mi][ni][v];
            if (a.relu) val = fmaxf(val, 0.f);
            a.y[(size_t)m * a.N + n] = val;
            if (a.amax_out) am.add(a.amax_out, m, val);
          }
        }
      }
    }
    if (a.amax_out)
      amax_commit_block<NT / 64>(a.amax_out, am.fb0, am.mx0, am.mx1, reinterpret_cast<float*>(smem));
  } else {
    // BN = 64 * HPB: heads nt*HPB .. nt*HPB + HPB - 1 (head_conv = 64 channels each);
    // per head: ReLU(conv3x3 + b) staged in LDS, then its 1x1 conv, channel-planar out
    static_assert(BN % 64 == 0, "whole heads per block");
    constexpr int HPB = BN / 64;
    float* T = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int hh = 0; hh < HPB; ++hh) {
      const int head = nt * HPB + hh;
      int ch = 0, hoff = 0;
#pragma unroll
      for (int j = 0; j < SFA_MAX_HEADS; ++j)
        if (j == head) {
          ch = a.hch[j];
          hoff = a.hoff[j];
        }
#pragma unroll
      for (int c0 = 0; c0 < BM; c0 += HCH) {
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int col = wn * WN + ni * 32 + r - 64 * hh;  // column within the head
          if (col < 0 || col >= 64) continue;
          const float bn = a.bias[n0 + 64 * hh + col];
          const float cs = PREC ? a.winv[n0 + 64 * hh + col] : 1.f;
#pragma unroll
          for (int mi = 0; mi < TM; ++mi)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
              const int row = wm * WM + mi * 32 + (v & 3) + 8 * (v >> 2) + 4 * h - c0;
              if (row >= 0 && row < HCH)
                T[row * 65 + col] = fmaxf((PREC ? acc[mi][ni][v] * rinv[mi][v] * cs : acc[mi][ni][v]) + bn, 0.f);
            }
        }
        __syncthreads();
        for (int idx = tid; idx < HCH * ch; idx += NT) {
          const int row = idx % HCH, c = idx / HCH;
          const int m = m0 + c0 + row;
          if (m >= M) continue;
          const float* wr = a.hw1 + (head * 4 + c) * 64;
          float s = a.hb1[head * 4 + c];
          const float* tr = T + row * 65;
#pragma unroll 16
          for (int k = 0; k < 64; ++k) s = fmaf(tr[k], wr[k], s);
          a.hout[(size_t)(hoff + c) * M + m] = s;
        }
        __syncthreads();
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int BK, int EPI, int OCC>
__global__ void __launch_bounds__((BM / WM) * (BN / WN) * 64, OCC) conv_x6_kernel(const ConvArgs a) {
  constexpr int NW = (BM / WM) * (BN / WN);
  constexpr int NT = NW * 64;
  constexpr int WAVES_N = BN / WN;
  static_assert(BK == 16 || BK == 32, "BK");
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int CPR = BK / 8;            // 16-B chunks per LDS row (per term)
  constexpr int KST = BK / 16;           // MFMA k-steps per tile
  // A loader: thread -> f32 quad kq of rows ar + ARPP*i
  constexpr int AQPR = BK / 4;
  constexpr int ARPP = NT / AQPR;
  constexpr int A_LD = BM / ARPP;
  static_assert(A_LD >= 1 && BM % ARPP == 0, "A loader");
  // B loader: thread -> 16-B chunk bc of rows br + BRPP*j, for each of the 3 terms
  constexpr int BRPP = NT / CPR;
  constexpr int B_LD = (BN + BRPP - 1) / BRPP;
  constexpr bool B_PART = BN % BRPP != 0;  // the last pass covers only rows < BN
  constexpr int ROWB = BK * 2;           // bytes per LDS row per term
  constexpr int TERM_A = BM * ROWB, TERM_B = BN * ROWB;
  constexpr int STAGE = 3 * (TERM_A + TERM_B);
  constexpr int HCH = BM < 128 ? BM : 128;
  constexpr int HEAD_BYTES = EPI == EPI_HEAD ? HCH * 65 * 4 : 0;
  constexpr int LDS_BYTES = 2 * STAGE > HEAD_BYTES ? 2 * STAGE : HEAD_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int n_tiles = a.N / BN;
  const int lbid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lbid / n_tiles, nt = lbid - mt * n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int M = a.M;

  auto swz = [](int row) { return BK == 16 ? ((row >> 3) & 1) : ((row >> 2) & 3); };

  const int kq = tid % AQPR, ar = tid / AQPR;
  constexpr int NSEG = 2;
  int r_ih[NSEG][A_LD], r_iw[NSEG][A_LD], r_pix[NSEG][A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int m = m0 + ar + ARPP * i;
    const bool ok = m < M;
    const int mm = ok ? m : 0;
    const int ow = mm % a.OW;
    const int t = mm / a.OW;
    const int oh = t % a.OH;
    const int b = t / a.OH;
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
      const ConvSeg& g = a.seg[sg];
      const int ih = oh * g.stride - g.pad;
      const int iw = ow * g.stride - g.pad;
      r_ih[sg][i] = ok ? ih : -(1 << 20);
      r_iw[sg][i] = iw;
      r_pix[sg][i] = (b * g.H + ih) * g.W + iw;
    }
  }
  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.seg[0].x), (short)0, (int)a.seg[0].bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.nseg > 1 ? a.seg[1].x : a.seg[0].x), (short)0,
      (int)(a.nseg > 1 ? a.seg[1].bytes : a.seg[0].bytes), 0x00020000);
  const unsigned term_bytes = (unsigned)a.N * (unsigned)a.Kpad * 2u;
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.wx), (short)0, (int)(3u * term_bytes), 0x00020000);

  const int bc = tid % CPR, br = tid / CPR;
  x6_f32x4 ra[A_LD];
  x6_u32x4 rb[3][B_LD];
  auto load_seg = [&](const int sg, const __amdgpu_buffer_rsrc_t rs, const int kl) {
    const ConvSeg& g = a.seg[sg];
    const int kk = kl + 4 * kq;
    const int tap = kk >> g.logC;
    const int c = kk & (g.C - 1);
    const int kh = (tap * g.kdiv_mul) >> g.kdiv_sh;
    const int kw = tap - kh * g.KW;
    const bool tap_ok = tap < g.taps;
    const int toff = kh * g.W + kw;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const bool ok = tap_ok & ((unsigned)(r_ih[sg][i] + kh) < (unsigned)g.H) &
                      ((unsigned)(r_iw[sg][i] + kw) < (unsigned)g.W);
      const unsigned off = ok ? (unsigned)((((r_pix[sg][i] + toff) << g.logC) + c) << 2) : 0x80000000u;
      ra[i] = __builtin_bit_cast(x6_f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  };
  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
    if (a.nseg > 1 && k0 >= a.kseg1)
      load_seg(1, rs1, k0 - a.kseg1);
    else
      load_seg(0, rs0, k0);
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      // rows past the tile read out of range -> zeros, never stored
      const bool in = !B_PART || br + BRPP * j < BN;
      const unsigned off = in ? (unsigned)(((n0 + br + BRPP * j) * a.Kpad + k0 + 8 * bc) << 1) : 0x80000000u;
#pragma unroll
      for (int t = 0; t < 3; ++t)
        rb[t][j] = __builtin_bit_cast(
            x6_u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsw, in ? off + t * term_bytes : off, 0, 0));
    }
  };
  auto store_tile = [&](int stage) {
    unsigned char* S = smem + stage * STAGE;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int R = ar + ARPP * i;
      const int byte = R * ROWB + (((kq >> 1) ^ swz(R)) << 4) + ((kq & 1) << 3);
      bf16x4_t t0, t1, t2;
      split3(ra[i], t0, t1, t2);
      *reinterpret_cast<bf16x4_t*>(S + byte) = t0;
      *reinterpret_cast<bf16x4_t*>(S + TERM_A + byte) = t1;
      *reinterpret_cast<bf16x4_t*>(S + 2 * TERM_A + byte) = t2;
    }
    unsigned char* SB = S + 3 * TERM_A;
#pragma unroll
    for (int j = 0; j < B_LD; ++j) {
      const int R = br + BRPP * j;
      if (B_PART && R >= BN) continue;
      const int byte = R * ROWB + ((bc ^ swz(R)) << 4);
#pragma unroll
      for (int t = 0; t < 3; ++t) *reinterpret_cast<x6_u32x4*>(SB + t * TERM_B + byte) = rb[t][j];
    }
  };

  x6_f32x16 acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[mi][ni][v] = 0.f;

  const int r = lane & 31, h = lane >> 5;
  auto compute = [&](int stage) {
    const unsigned char* S = smem + stage * STAGE;
    const unsigned char* SB = S + 3 * TERM_A;
#pragma unroll
    for (int s = 0; s < KST; ++s) {
      bf16x8_t af[3][TM], bf[3][TN];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const int R = wm * WM + mi * 32 + r;
        const int byte = R * ROWB + (((2 * s + h) ^ swz(R)) << 4);
#pragma unroll
        for (int t = 0; t < 3; ++t) af[t][mi] = *reinterpret_cast<const bf16x8_t*>(S + t * TERM_A + byte);
      }
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int R = wn * WN + ni * 32 + r;
        const int byte = R * ROWB + (((2 * s + h) ^ swz(R)) << 4);
#pragma unroll
        for (int t = 0; t < 3; ++t) bf[t][ni] = *reinterpret_cast<const bf16x8_t*>(SB + t * TERM_B + byte);
      }
      // smallest terms first
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          x6_f32x16 c = acc[mi][ni];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2][mi], bf[0][ni], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][mi], bf[2][ni], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][mi], bf[1][ni], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][mi], bf[0][ni], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][mi], bf[1][ni], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][mi], bf[0][ni], c, 0, 0, 0);
          acc[mi][ni] = c;
        }
    }
  };

  const int nk = a.Kpad / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    load_tile(kt + 1 < nk ? kt + 1 : kt);
    compute(cur);
    store_tile(cur ^ 1);
    __syncthreads();
  }

  const float one[TM] = {};
  x6_epilogue<BM, BN, WM, WN, TM, TN, NT, EPI>(a, acc, smem, m0, n0, nt, wm, wn, tid, one);
}

// LDS-DMA variant: A (f32) and the three W terms (bf16) stream into an NSTAGE-deep
// ring with buffer_load ... lds (no VGPR staging); A is split into its bf16 terms when a
// wave reads its fragment.  Waves are stacked along M only (WN = BN), so every A
// element is split exactly once.  LDS images (16-B quad/chunk q of row R stored at
// q ^ swz(R), conflict-free for the ds_read_b128 lane groups):
//   A rows BK f32: 64 B (BK 16, swz = (R >> 2) & 3) or 128 B (BK 32, swz = (R >> 1) & 7)
//   W rows BK bf16 per term: 32 B (BK 16, swz = (R >> 3) & 1) or 64 B (BK 32, (R >> 2) & 3)
// DMA instructions (1 KiB each) are dealt round-robin to the waves; each wave waits for
// its own with a counted vmcnt, then the barrier makes the whole stage visible.
// ABL: diagnostic ablation bits for tools/convbench (0 in the product): 1 = no DMA in
// the K loop, 2 = no A split (raw bits as terms), 4 = W fragments read once per k-step
// group instead of per column block, 8 = no barrier, 16 = no epilogue (one sum per lane
// stored), 64 = s_setprio 1 for the second half of the waves (the SIMD partners).
// PREC 1: the fp16x3 form (two fp16 W terms, scaled A split into two fp16 terms when read,
// products hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_f16).
template <int BM, int BN, int WM, int EPI, int OCC, int BK = 16, int NSTAGE = 3, int ABL = 0,
          int WNT = BN, int PREC = 0>
__global__ void __launch_bounds__((BM / WM) * (BN / WNT) * 64, OCC) conv_x6g_kernel(const ConvArgs a) {
  static_assert(BK == 16 || BK == 32, "BK");
  static_assert(NSTAGE == 2 || NSTAGE == 3, "ring depth");
  constexpr int WN = WNT;                 // BN: waves along M only (A split once)
  constexpr int WAVES_N = BN / WN;
  constexpr int NW = (BM / WM) * WAVES_N;
  constexpr int NT = NW * 64;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int KST = BK / 16;
  constexpr int AROW = BK * 4, BROW = BK * 2;         // bytes per LDS row
  constexpr int NTW = PREC ? 2 : 3;                   // W terms
  constexpr int A_BYTES = BM * AROW, TERM_B = BN * BROW;
  constexpr int STAGE = A_BYTES + NTW * TERM_B;
  constexpr int A_RPD = 1024 / AROW, B_RPD = 1024 / BROW;  // rows per DMA instruction
  constexpr int ND_A = BM / A_RPD;
  constexpr int ND_BT = BN / B_RPD;                         // per term
  constexpr int ND = ND_A + NTW * ND_BT;
  constexpr int DPW = (ND + NW - 1) / NW;  // max per wave
  constexpr int DREM = ND % NW;            // waves < DREM issue DPW, the rest DPW - 1 (if DREM)
  static_assert(BM % A_RPD == 0 && BN % B_RPD == 0 && BN % 32 == 0, "tile");
  constexpr int HCH = BM < 128 ? BM : 128;
  constexpr int HEAD_BYTES = EPI == EPI_HEAD ? HCH * 65 * 4 : 0;
  constexpr int LDS_BYTES = NSTAGE * STAGE > HEAD_BYTES ? NSTAGE * STAGE : HEAD_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];

  auto swzA = [](int R) { return BK == 16 ? ((R >> 2) & 3) : ((R >> 1) & 7); };
  auto swzB = [](int R) { return BK == 16 ? ((R >> 3) & 1) : ((R >> 2) & 3); };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar DMA bookkeeping
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int n_tiles = a.N / BN;
  const int lbid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lbid / n_tiles, nt = lbid - mt * n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int M = a.M;

  // this wave's A DMA instructions: d = wave + NW * i (d < ND_A); lane -> row, quad
  constexpr int QPR = AROW / 16;
  const int arow_in = lane / QPR;
  // logical f32 quad of this lane: the same for all of the wave's A instructions, since
  // rows A_RPD*(wave + NW*i) + arow_in share swzA (BK 16: A_RPD = 16; BK 32: NW even)
  static_assert(BK == 16 || NW % 2 == 0, "swizzle period");
  const int kq = (lane % QPR) ^ swzA(A_RPD * wave + arow_in);
  constexpr int NSEG = 2;
  int r_ih[NSEG][DPW], r_iw[NSEG][DPW], r_pix[NSEG][DPW];
#pragma unroll
  for (int i = 0; i < DPW; ++i) {
    const int d = wave + NW * i;
    const int R = A_RPD * d + arow_in;           // A row (valid when d < ND_A)
    const int m = m0 + R;
    const bool ok = d < ND_A && m < M;
    const int mm = ok ? m : 0;
    const int ow = mm % a.OW;
    const int t = mm / a.OW;
    const int oh = t % a.OH;
    const int b = t / a.OH;
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
      const ConvSeg& g = a.seg[sg];
      const int ih = oh * g.stride - g.pad;
      const int iw = ow * g.stride - g.pad;
      r_ih[sg][i] = ok ? ih : -(1 << 20);
      r_iw[sg][i] = iw;
      r_pix[sg][i] = (b * g.H + ih) * g.W + iw;
    }
  }
  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.seg[0].x), (short)0, (int)a.seg[0].bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.nseg > 1 ? a.seg[1].x : a.seg[0].x), (short)0,
      (int)(a.nseg > 1 ? a.seg[1].bytes : a.seg[0].bytes), 0x00020000);
  const unsigned term_bytes = (unsigned)a.N * (unsigned)a.Kpad * 2u;
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(PREC ? a.wh : a.wx), (short)0, (int)(NTW * term_bytes), 0x00020000);
  // fp16x3: per A row (this lane's row of each 32-row MFMA tile) the scale of its frame
  float as[TM], ainv[TM];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    as[mi] = ainv[mi] = 1.f;
    if constexpr (PREC == 1) {
      const int m = min(m0 + wm * WM + mi * 32 + (lane & 31), M - 1);
      as[mi] = amax_frame_scale(a.amax_in, a.nseg, m / (a.OH * a.OW), ainv[mi]);
    }
  }
  // W lanes: row brow_in of the instruction's B_RPD rows, chunk (lane % CPR)
  constexpr int CPR = BROW / 16;
  const int brow_in = lane / CPR;

  // A DMAs of one K-tile from segment SG (compile-time, so the buffer resource and
  // the per-row window origins stay in SGPRs / VGPRs — no waterfall, no scratch)
  auto load_a = [&](auto sgc, const __amdgpu_buffer_rsrc_t rs, int kl, unsigned char* S) {
    constexpr int SG = decltype(sgc)::value;
    const ConvSeg& g = a.seg[SG];
    const int kk = kl + 4 * kq;
    const int tap = kk >> g.logC;
    const int c = kk & (g.C - 1);
    const int kh = (tap * g.kdiv_mul) >> g.kdiv_sh;
    const int kw = tap - kh * g.KW;
    const bool tap_ok = tap < g.taps;
    const int toff = kh * g.W + kw;
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int d = wave + NW * i;
      if (d < ND_A) {
        const bool ok = tap_ok & ((unsigned)(r_ih[SG][i] + kh) < (unsigned)g.H) &
                        ((unsigned)(r_iw[SG][i] + kw) < (unsigned)g.W);
        const unsigned off = ok ? (unsigned)((((r_pix[SG][i] + toff) << g.logC) + c) << 2) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(S + d * 1024),
                                                 16, off, 0, 0, 0);
      }
    }
  };
  auto load_tile = [&](int kt, unsigned char* S) {
    const int k0 = kt * BK;
    if (a.nseg > 1 && k0 >= a.kseg1)
      load_a(std::integral_constant<int, 1>(), rs1, k0 - a.kseg1, S);
    else
      load_a(std::integral_constant<int, 0>(), rs0, k0, S);
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int d = wave + NW * i;
      if (d >= ND_A && d < ND) {
        const int e = d - ND_A;
        const int t = e / ND_BT;
        const int R = (e % ND_BT) * B_RPD + brow_in;
        const int lc = (lane % CPR) ^ swzB(R);
        const unsigned off = t * term_bytes + (unsigned)(((n0 + R) * a.Kpad + k0 + 8 * lc) << 1);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsw, (__attribute__((address_space(3))) void*)(S + A_BYTES + e * 1024), 16, off, 0, 0, 0);
      }
    }
  };

  x6_f32x16 acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[mi][ni][v] = 0.f;

  const int r = lane & 31, h = lane >> 5;
  auto compute = [&](const unsigned char* S) {
    const unsigned char* SB = S + A_BYTES;
#pragma unroll
    for (int s = 0; s < KST; ++s) {
      if constexpr (PREC == 1) {
        f16x8_t hf[2][TM];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          const int R = wm * WM + mi * 32 + r;
          const int q = 4 * s + 2 * h;
          const x6_f32x4 q0 = *reinterpret_cast<const x6_f32x4*>(S + R * AROW + ((q ^ swzA(R)) << 4));
          const x6_f32x4 q1 = *reinterpret_cast<const x6_f32x4*>(S + R * AROW + (((q + 1) ^ swzA(R)) << 4));
          f16x4_t t0, t1, u0, u1;
          split2h(q0, as[mi], t0, t1);
          split2h(q1, as[mi], u0, u1);
          hf[0][mi] = __builtin_shufflevector(t0, u0, 0, 1, 2, 3, 4, 5, 6, 7);
          hf[1][mi] = __builtin_shufflevector(t1, u1, 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int R = wn * WN + ni * 32 + r;
          const int byte = R * BROW + (((2 * s + h) ^ swzB(R)) << 4);
          const f16x8_t b0 = *reinterpret_cast<const f16x8_t*>(SB + byte);
          const f16x8_t b1 = *reinterpret_cast<const f16x8_t*>(SB + TERM_B + byte);
#pragma unroll
          for (int mi = 0; mi < TM; ++mi) {
            x6_f32x16 c = acc[mi][ni];
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(hf[1][mi], b0, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(hf[0][mi], b1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(hf[0][mi], b0, c, 0, 0, 0);
            acc[mi][ni] = c;
          }
        }
        continue;
      }
      bf16x8_t af[3][TM];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const int R = wm * WM + mi * 32 + r;
        const int q = 4 * s + 2 * h;  // logical f32 quads q, q + 1 hold k = 16s + 8h .. + 7
        const x6_f32x4 q0 = *reinterpret_cast<const x6_f32x4*>(S + R * AROW + ((q ^ swzA(R)) << 4));
        const x6_f32x4 q1 = *reinterpret_cast<const x6_f32x4*>(S + R * AROW + (((q + 1) ^ swzA(R)) << 4));
        if constexpr (ABL & 2) {
          const bf16x8_t raw = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(
                                                               __builtin_bit_cast(x6_u32x4, q0), __builtin_bit_cast(x6_u32x4, q1), 0, 2, 4, 6));
          af[0][mi] = raw;
          af[1][mi] = raw;
          af[2][mi] = raw;
        } else {
          bf16x4_t t0, t1, t2, u0, u1, u2;
          split3(q0, t0, t1, t2);
          split3(q1, u0, u1, u2);
          af[0][mi] = __builtin_shufflevector(t0, u0, 0, 1, 2, 3, 4, 5, 6, 7);
          af[1][mi] = __builtin_shufflevector(t1, u1, 0, 1, 2, 3, 4, 5, 6, 7);
          af[2][mi] = __builtin_shufflevector(t2, u2, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int R = ((ABL & 4) ? 0 : wn * WN + ni * 32) + r;
        const int byte = R * BROW + (((2 * s + h) ^ swzB(R)) << 4);
        bf16x8_t b0 = *reinterpret_cast<const bf16x8_t*>(SB + byte);
        bf16x8_t b1 = *reinterpret_cast<const bf16x8_t*>(SB + TERM_B + byte);
        bf16x8_t b2 = *reinterpret_cast<const bf16x8_t*>(SB + 2 * TERM_B + byte);
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          x6_f32x16 c = acc[mi][ni];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2][mi], b0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][mi], b2, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][mi], b1, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][mi], b0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][mi], b1, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][mi], b0, c, 0, 0, 0);
          acc[mi][ni] = c;
        }
      }
    }
  };

  const int nk = a.Kpad / BK;
  if constexpr ((ABL & 64) != 0) {
    if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }
  if constexpr (NSTAGE == 3) {
    load_tile(0, smem);
    load_tile(nk > 1 ? 1 : 0, smem + STAGE);
    for (int kt = 0; kt < nk; ++kt) {
      // this wave's DMAs of tile kt have landed (those of kt + 1 may be in flight)
      if (DREM == 0 || wave < DREM)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPW) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPW - 1) : "memory");
      if constexpr (!(ABL & 8)) __builtin_amdgcn_s_barrier();  // ... and every wave's: stage kt % 3 is complete
      if constexpr (!(ABL & 1)) load_tile(kt + 2 < nk ? kt + 2 : nk - 1, smem + ((kt + 2) % 3) * STAGE);
      compute(smem + (kt % 3) * STAGE);
    }
  } else {
    load_tile(0, smem);
    for (int kt = 0; kt < nk; ++kt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile kt landed (this wave)
      if constexpr (!(ABL & 8)) __builtin_amdgcn_s_barrier();  // every wave: stage kt & 1 complete, stage (kt+1) & 1 free
      if constexpr (!(ABL & 1)) load_tile(kt + 1 < nk ? kt + 1 : nk - 1, smem + ((kt + 1) & 1) * STAGE);
      compute(smem + (kt & 1) * STAGE);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr ((ABL & 16) != 0) {
    float t = 0.f;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int v = 0; v < 16; ++v) t += acc[mi][ni][v];
    a.y[(size_t)blockIdx.x * NT + tid] = t;
    return;
  }
  __syncthreads();
  x6_epilogue<BM, BN, WM, WN, TM, TN, NT, EPI, PREC>(a, acc, smem, m0, n0, nt, wm, wn, tid, ainv);
}

template <int BM, int BN, int WM, int EPI, int OCC, int BK = 16, int NSTAGE = 3, int ABL = 0,
          int WNT = BN, int PREC = 0>
inline int launch_conv_x6g_cfg(const ConvArgs& a, hipStream_t st) {
  if (!(PREC ? a.wh != nullptr && a.winv != nullptr : a.wx != nullptr) || a.Kpad % BK != 0 || (a.nseg == 2 && a.kseg1 % BK != 0) || a.N % BN != 0) {
    set_error("conv_x6g: K/N not aligned to the tile or no split weights (Kpad=%d kseg1=%d N=%d)",
              a.Kpad, a.kseg1, a.N);
    return SFA_E_UNSUPPORTED;
  }
  if (3ull * a.N * a.Kpad * 2ull >= (1ull << 31)) {
    set_error("conv_x6g: split weights >= 2 GiB");
    return SFA_E_UNSUPPORTED;
  }
  const long long nblocks = (long long)ceil_div(a.M, BM) * (a.N / BN);
  if (nblocks <= 0 || nblocks > 0x7fffffffll) {
    set_error("conv_x6g: bad grid (M=%d N=%d)", a.M, a.N);
    return SFA_E_INVALID;
  }
  hipLaunchKernelGGL((conv_x6g_kernel<BM, BN, WM, EPI, OCC, BK, NSTAGE, ABL, WNT, PREC>),
                     dim3((unsigned)nblocks), dim3((BM / WM) * (BN / WNT) * 64), 0, st, a);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

template <int BM, int BN, int WM, int WN, int BK, int EPI, int OCC>
inline int launch_conv_x6_cfg(const ConvArgs& a, hipStream_t st) {
  if (!a.wx || a.Kpad % BK != 0 || (a.nseg == 2 && a.kseg1 % BK != 0) || a.N % BN != 0) {
    set_error("conv_x6: K/N not aligned to the tile or no split weights (Kpad=%d kseg1=%d N=%d)",
              a.Kpad, a.kseg1, a.N);
    return SFA_E_UNSUPPORTED;
  }
  if (3ull * a.N * a.Kpad * 2ull >= (1ull << 31)) {
    set_error("conv_x6: split weights >= 2 GiB");
    return SFA_E_UNSUPPORTED;
  }
  const int mt = ceil_div(a.M, BM);
  const long long nblocks = (long long)mt * (a.N / BN);
  if (nblocks <= 0 || nblocks > 0x7fffffffll) {
    set_error("conv_x6: bad grid (M=%d N=%d)", a.M, a.N);
    return SFA_E_INVALID;
  }
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  hipLaunchKernelGGL((conv_x6_kernel<BM, BN, WM, WN, BK, EPI, OCC>), dim3((unsigned)nblocks), dim3(NT),
                     0, st, a);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

}  // namespace sfa
