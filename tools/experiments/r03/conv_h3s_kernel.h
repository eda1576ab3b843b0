// 3x3 / stride-1 / pad-1 implicit-GEMM convolution, fp16x3 on v_mfma_f32_16x16x32_f16, with the
// A operand staged ONCE per (kh, 32-channel chunk) as a row strip shared by the three kw taps.
// conv_h3_kernel stages A once per tap: three times the LDS-DMA pieces for it, and an LDS-DMA
// piece costs ~60 issue cycles among MFMAs (MI355X_MICROARCH.md cycle table).
//
// Strip row j of a block holds the input pixel (y(m) + kh - 1, x(m)) of output row m = m0 - 1 + j
// (32 channels, f32).  Output row m at tap kw reads strip row (m - m0) + kw, the pixel of output
// m + kw - 1: the right one whenever x(m) + kw - 1 lies inside the image row (then m + kw - 1 is
// in the same row), and otherwise the conv's zero padding, which the fragment read applies by
// zeroing rows with x(m) == 0 (kw 0) or x(m) == W - 1 (kw 2).  Rows above or below the image
// load zeros (out-of-range buffer offset).  The fp16x3 split, the swizzles, W staging, split-K
// and the epilogues are conv_h3_kernel<..., MF = 1>'s.
// LDS: two strip buffers ((BM + 2) x 128 B in 1-KiB DMA pieces) and two W stages.  Per k-step
// (one kw): wait for W(t) (at kw 0 also the strip), barrier, issue W(t + 1) (at kw 0 also the
// next strip), compute.  Counted vmcnt: kw 0 and 2 -> 0; kw 1 -> the wave's strip pieces, issued
// after W(t).  The last step re-issues its own tiles, so the counts stay uniform.
#pragma once

#include "conv_r3_kernel.h"

namespace sfa {

// ABL: 1 = no fp16x3 split (the f32 bits are fed to the MFMAs; convbench ablation only),
// 32 = no epilogue, 64 = no pre-split VALU (ablations, results wrong), 128 = (with 4 and 2) the
// residual tile loaded at the last super-step's kw 1 (in place of the no-op strip reload), so
// the last six k-steps' MFMAs hide its latency, 256 / 512 = epilogue without stores / without
// the amax record (ablations), 1024 = (with 2) output tile staged in LDS and stored
// row-contiguous (whole 128-B lines per store instruction), 2048 = non-temporal output stores,
// 2 = transposed accumulators (W fragment as the MFMA A operand) with conv_r3_kernel.h's float4
// epilogue (r3t_epilogue_std) and float4 split-K partials,
// 4 = pre-split strip: at kw 0 each wave splits ITS rows of the f32 strip (WM + 2 rows, the kw
// halo included) once into fp16 hi / lo rows of a private LDS region, and the three kw k-steps
// read ready fp16 fragments (a third of the split VALU; conv padding by reading a zero row).
// One f32 strip buffer: the next strip is issued at kw 1, when every wave has split this one.
// 8 = fp16 split in 2 VALU per value (split2h_x8 / split2h_pair, inline v_fma_mix),
// 16 = spread DMA: the k-step's W pieces (and the strip pieces, when due) are issued between the
// MFMAs of column blocks 1, 2, .. (W first, then the strip: the counted waits are unchanged)
// instead of in a burst right after the barrier.
// 4096 = no W DMA inside the K loop (the first k-step's W is reused; ablation of the W staging
// latency, results wrong), 8192 = the W DMA issued as usual but never waited for (its latency
// hidden, its issue and traffic kept; ablation, results wrong),
// 16384 = A prefetch: the fragments of tap kw + 1 (same strip) are read and split during tap kw's
// MFMAs (after column block TN / 2), so a k-step's first MFMAs wait only for their W fragments.
template <int BM, int BN, int WM, int EPI, int OCC, int ABL = 0>
__global__ void __launch_bounds__((BM / WM) * 64, OCC) conv_h3s_kernel(const ConvArgs a) {
  constexpr int NW = BM / WM, NT = NW * 64;
  constexpr int TM = WM / 16, TN = BN / 16;
  constexpr int AROW = 128, BROW = 64;  // bytes per LDS row: 32 f32 / 32 fp16
  constexpr int SROWS = BM + 2;          // strip rows m0 - 1 .. m0 + BM
  constexpr int ND_S = (SROWS + 7) / 8;  // strip DMA pieces (8 rows each)
  constexpr int S_BYTES = ND_S * 1024;
  constexpr int TERM_B = BN * BROW, W_BYTES = 2 * TERM_B;
  constexpr int ND_B = W_BYTES / 1024;  // W pieces per k-step (16 rows each)
  constexpr int NS = (ND_S + NW - 1) / NW, NS_REM = ND_S % NW;
  constexpr int NB = (ND_B + NW - 1) / NW, NB_REM = ND_B % NW;
  constexpr int HEAD_BYTES = EPI == EPI_HEAD ? BM * 65 * 4 + (BN / 64) * 1024 : 0;  // h3_epilogue16
  constexpr bool PS = (ABL & 4) != 0;
  constexpr bool RESPF = PS && (ABL & 128) != 0 && (ABL & 2) != 0 && (ABL & 16) == 0;
  constexpr int PROWS = WM + 2;              // a wave's pre-split rows (its WM rows + the kw halo)
  constexpr int PR_BYTES = (PROWS + 1) * 64;  // per term: 32 fp16 per row, + one zero row
  constexpr int NSB = PS ? 1 : 2;             // f32 strip buffers
  constexpr int MAIN_BYTES = NSB * S_BYTES + 2 * W_BYTES + (PS ? NW * 2 * PR_BYTES : 0);
  constexpr bool STG = (ABL & 1024) != 0 && (ABL & 2) != 0 && EPI == EPI_STD;  // row-contiguous stores via LDS
  constexpr int STG_BYTES = STG ? r3t_stage_bytes<TM, TN, NT>() : 0;
  constexpr int LDS_BYTES0 = MAIN_BYTES > HEAD_BYTES ? MAIN_BYTES : HEAD_BYTES;
  constexpr int LDS_BYTES = LDS_BYTES0 > STG_BYTES ? LDS_BYTES0 : STG_BYTES;
  static_assert(NW % 2 == 0 && WM % 16 == 0 && BN % 16 == 0, "tile");
  static_assert((ABL & 2) == 0 || EPI == EPI_STD, "transposed form: standard epilogue only");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];

  auto swzA = [](int R) { return ((R >> 1) & 7) ^ ((((R & 15) + 4) >> 2) & 2); };
  auto swzB = [](int R) { return ((R >> 2) & 3) ^ ((((R & 15) + 4) >> 3) & 1); };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_tiles = a.N / BN, m_tiles = (a.M + BM - 1) / BM;
  const int nsplit = a.ksplit > 1 ? a.ksplit : 1;
  int lbid = xcd_remap(blockIdx.x, gridDim.x);
  const int kz = lbid / (m_tiles * n_tiles);  // split-K slice
  lbid -= kz * (m_tiles * n_tiles);
  const int mt = lbid / n_tiles, nt = lbid - mt * n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int M = a.M;
  const ConvSeg& g = a.seg[0];
  const int H = g.H, W = g.W;

  // strip pieces d = wave + NW * i: rows 8d + lane / 8 (d of the wave's parity: one swizzle)
  const int srow = lane >> 3;
  const int kq = (lane & 7) ^ swzA(8 * wave + srow);
  int s_pix[NS], s_y[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const int j = 8 * (wave + NW * i) + srow;
    const int m = m0 - 1 + j;
    const bool ok = j < SROWS && m >= 0 && m < M;
    const int mm = ok ? m : 0;
    const int x = mm % W, t = mm / W;
    const int y = t % H, b = t / H;
    s_pix[i] = (b * H + y) * W + x;
    s_y[i] = ok ? y : -(1 << 20);
  }
  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.x), (short)0, (int)g.bytes, 0x00020000);
  const unsigned term_bytes = (unsigned)a.N * (unsigned)a.Kpad * 2u;
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.wh), (short)0,
                                                                       (int)(2 * term_bytes), 0x00020000);
  int boff[NB];  // int + unsigned cast at the use (see conv_h3_kernel)
#pragma unroll
  for (int jj = 0; jj < NB; ++jj) {
    const int e = wave + NW * jj < ND_B ? wave + NW * jj : ND_B - 1;
    const int term = e / (ND_B / 2);
    const int R = (e - term * (ND_B / 2)) * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ swzB(R);
    boff[jj] = (int)(term * term_bytes) + (int)(((n0 + R) * a.Kpad + 8 * lc) << 1);
  }
  // x of this lane's A row in each 16-row tile (kw edge masks); its frame's fp16x3 scale
  const int c16 = lane & 15, gq = lane >> 4;
  int xm[TM];
  float as[TM], ainv[TM];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    const int m = min(m0 + wave * WM + mi * 16 + c16, M - 1);
    xm[mi] = m % W;
    as[mi] = amax_frame_scale(a.amax_in, 1, m / (a.OH * a.OW), ainv[mi]);
  }

  // pre-split (PS): scale of strip row j = the frame of output row m0 - 1 + j (a block spans at
  // most two frames; rows of another frame than their consumer are always masked as padding)
  const int P = a.OH * a.OW;
  const int fb = (m0 / P + 1) * P;  // first row of the next frame
  float sA = 1.f, sB = 1.f;
  if constexpr (PS) {
    float t;
    sA = amax_frame_scale(a.amax_in, 1, m0 / P, t);
    sB = fb < M ? amax_frame_scale(a.amax_in, 1, fb / P, t) : sA;
  }
  auto swzP = [](int R) { return ((R >> 2) & 1) << 1; };  // conflict-free at every kw row offset

  const int nchunk = g.C >> 5;
  const int nsl = 3 * nchunk / nsplit;  // this block's (kh, chunk) super-steps s0 .. s0 + nsl - 1
  const int s0 = kz * nsl;
  auto load_strip = [&](int s, unsigned char* S) {
    const int kh = s / nchunk, c0 = (s - kh * nchunk) << 5;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      if (NS_REM == 0 || i < NS - 1 || wave < NS_REM) {
        const bool ok = (unsigned)(s_y[i] + kh - 1) < (unsigned)H;
        const unsigned off =
            ok ? (unsigned)((((s_pix[i] + (kh - 1) * W) << g.logC) + c0 + 4 * kq) << 2) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsx, (__attribute__((address_space(3))) void*)(S + (wave + NW * i) * 1024), 16, off, 0, 0, 0);
      }
    }
  };
  auto load_strip_piece = [&](int i, int s, unsigned char* S) {
    const int kh = s / nchunk, c0 = (s - kh * nchunk) << 5;
    if (NS_REM == 0 || i < NS - 1 || wave < NS_REM) {
      const bool ok = (unsigned)(s_y[i] + kh - 1) < (unsigned)H;
      const unsigned off =
          ok ? (unsigned)((((s_pix[i] + (kh - 1) * W) << g.logC) + c0 + 4 * kq) << 2) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsx, (__attribute__((address_space(3))) void*)(S + (wave + NW * i) * 1024), 16, off, 0, 0, 0);
    }
  };
  auto load_w_piece = [&](int jj, int k0, unsigned char* S) {
    if constexpr ((ABL & 4096) != 0) return;
    if (NB_REM == 0 || jj < NB - 1 || wave < NB_REM)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsw, (__attribute__((address_space(3))) void*)(S + (wave + NW * jj) * 1024), 16,
          (unsigned)(boff[jj] + 2 * k0), 0, 0, 0);
  };
  bool w_in_loop = false;  // ABL 4096: only the prologue's W DMA
  auto load_w = [&](int k0, unsigned char* S) {
#pragma unroll
    for (int jj = 0; jj < NB; ++jj) {
      if ((ABL & 4096) != 0 && w_in_loop) break;
      if (NB_REM == 0 || jj < NB - 1 || wave < NB_REM)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsw, (__attribute__((address_space(3))) void*)(S + (wave + NW * jj) * 1024), 16,
            (unsigned)(boff[jj] + 2 * k0), 0, 0, 0);
    }
  };
  auto wk0 = [&](int s, int kw) {  // K offset of the W tile of super-step s, tap kw
    const int kh = s / nchunk, c0 = (s - kh * nchunk) << 5;
    return (kh * 3 + kw) * g.C + c0;
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[mi][ni][v] = 0.f;
  x6_f32x4 rvp[TM][TN];  // RESPF: the residual tile, loaded during the last super-step

  unsigned char* const PH = smem + NSB * S_BYTES + 2 * W_BYTES + wave * 2 * PR_BYTES;  // PS: hi rows, lo + PR_BYTES
  auto presplit = [&](const unsigned char* Ss) {
    const int rr = lane >> 3, q = lane & 7;
#pragma unroll
    for (int p = 0; p < (PROWS + 7) / 8; ++p) {
      const int r = 8 * p + rr;
      if (r < PROWS) {
        const int j = wave * WM + r;
        const x6_f32x4 x = *reinterpret_cast<const x6_f32x4*>(Ss + j * AROW + ((q ^ swzA(j)) << 4));
        const float sc = m0 - 1 + j >= fb ? sB : sA;
        const int off = r * 64 + (((q >> 1) ^ swzP(r)) << 4) + (q & 1) * 8;
        if constexpr ((ABL & 64) != 0) {  // ablation: no split VALU (raw bits stored)
          typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
          const u32x2_t raw = u32x2_t{__float_as_uint(x[0]) ^ __float_as_uint(x[1]), __float_as_uint(x[2])};
          *reinterpret_cast<u32x2_t*>(PH + off) = raw;
          *reinterpret_cast<u32x2_t*>(PH + PR_BYTES + off) = raw;
        } else if constexpr ((ABL & 8) != 0) {
          typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
          unsigned h0, h1, l0, l1;
          split2h_pair(x[0], x[1], sc, h0, l0);
          split2h_pair(x[2], x[3], sc, h1, l1);
          *reinterpret_cast<u32x2_t*>(PH + off) = u32x2_t{h0, h1};
          *reinterpret_cast<u32x2_t*>(PH + PR_BYTES + off) = u32x2_t{l0, l1};
        } else {
          f16x4_t hi, lo;
          split2h(x, sc, hi, lo);
          *reinterpret_cast<f16x4_t*>(PH + off) = hi;
          *reinterpret_cast<f16x4_t*>(PH + PR_BYTES + off) = lo;
        }
      }
    }
  };
  if constexpr (PS) {  // the zero rows (conv padding at kw 0 / 2)
    if (lane < 8) *reinterpret_cast<x6_f32x4*>(PH + (lane & 4 ? PR_BYTES : 0) + PROWS * 64 + (lane & 3) * 16) =
        x6_f32x4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr bool APF = (ABL & 16384) != 0;
  f16x8_t hfn[2][TM];  // APF: the next tap's split A fragments
  auto read_a = [&](const unsigned char* Ss, int kw, f16x8_t (&hf)[2][TM]) {
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      if constexpr (PS) {
        const bool pad = kw == 0 ? xm[mi] == 0 : (kw == 2 ? xm[mi] == W - 1 : false);
        const int R = pad ? PROWS : mi * 16 + c16 + kw;
        const int o = R * 64 + ((gq ^ swzP(R)) << 4);
        hf[0][mi] = *reinterpret_cast<const f16x8_t*>(PH + o);
        hf[1][mi] = *reinterpret_cast<const f16x8_t*>(PH + PR_BYTES + o);
        continue;
      }
      const int R = wave * WM + mi * 16 + c16 + kw;
      x6_f32x4 q0 = *reinterpret_cast<const x6_f32x4*>(Ss + R * AROW + (((2 * gq) ^ swzA(R)) << 4));
      x6_f32x4 q1 = *reinterpret_cast<const x6_f32x4*>(Ss + R * AROW + (((2 * gq + 1) ^ swzA(R)) << 4));
      const bool pad = kw == 0 ? xm[mi] == 0 : (kw == 2 ? xm[mi] == W - 1 : false);
      if (pad) {
        q0 = x6_f32x4{0.f, 0.f, 0.f, 0.f};
        q1 = q0;
      }
      if constexpr ((ABL & 1) != 0) {
        hf[0][mi] = __builtin_bit_cast(f16x8_t, __builtin_shufflevector(q0, q0, 0, 1, 2, 3));
        hf[1][mi] = __builtin_bit_cast(f16x8_t, __builtin_shufflevector(q1, q1, 0, 1, 2, 3));
      } else if constexpr ((ABL & 8) != 0) {
        split2h_x8(q0, q1, as[mi], hf[0][mi], hf[1][mi]);
      } else {
        f16x4_t t0, t1, u0, u1;
        split2h(q0, as[mi], t0, t1);
        split2h(q1, as[mi], u0, u1);
        hf[0][mi] = __builtin_shufflevector(t0, u0, 0, 1, 2, 3, 4, 5, 6, 7);
        hf[1][mi] = __builtin_shufflevector(t1, u1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
  };
  auto compute = [&](const unsigned char* Ss, const unsigned char* Sw, int kw, auto&& issue) {
    f16x8_t hf[2][TM];
    if (APF && kw > 0) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        hf[0][mi] = hfn[0][mi];
        hf[1][mi] = hfn[1][mi];
      }
    } else {
      read_a(Ss, kw, hf);
    }
    const unsigned char* SB = Sw + c16 * BROW + ((gq ^ swzB(c16)) << 4);
    f16x8_t bq[3][2];
    auto read_b = [&](int ni) {
      bq[ni % 3][0] = *reinterpret_cast<const f16x8_t*>(SB + ni * 16 * BROW);
      bq[ni % 3][1] = *reinterpret_cast<const f16x8_t*>(SB + TERM_B + ni * 16 * BROW);
    };
    read_b(0);
    if (TN > 1) read_b(1);
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      issue(ni);
      if (ni + 2 < TN) read_b(ni + 2);
      if (APF && kw < 2 && ni == TN / 2) read_a(Ss, kw + 1, hfn);
      const f16x8_t c0 = bq[ni % 3][0], c1 = bq[ni % 3][1];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        f32x4_t cc = acc[mi][ni];
        if constexpr ((ABL & 2) != 0) {
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[1][mi], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c1, hf[0][mi], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[0][mi], cc, 0, 0, 0);
        } else {
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(hf[1][mi], c0, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(hf[0][mi], c1, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(hf[0][mi], c0, cc, 0, 0, 0);
        }
        acc[mi][ni] = cc;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // SPREAD: the pieces of a k-step, W first, then (when due) the strip, dealt over column blocks
  // 1 .. TN - 1, PPB per block
  constexpr bool SPREAD = (ABL & 16) != 0;
  static_assert(!SPREAD || TN >= 2, "spread DMA needs two column blocks");
  auto spread_issue = [&](int ni, bool with_strip, int wk, unsigned char* wdst, int snext, unsigned char* sdst) {
    if (ni == 0) return;
    constexpr int PPB_W = (NB + NS + TN - 2) / (TN - 1);  // pieces per block when the strip is due
    constexpr int PPB_N = (NB + TN - 2) / (TN - 1);       // W only
#pragma unroll
    for (int u = 0; u < PPB_W; ++u) {
      const int ppb = with_strip ? PPB_W : PPB_N;
      if (u >= ppb) break;
      const int pidx = (ni - 1) * ppb + u;
      if (pidx < NB)
        load_w_piece(pidx, wk, wdst);
      else if (with_strip && pidx < NB + NS)
        load_strip_piece(pidx - NB, snext, sdst);
    }
  };
  unsigned char* const WB = smem + NSB * S_BYTES;
  load_strip(s0, smem);
  load_w(wk0(s0, 0), WB);
  w_in_loop = true;
  constexpr int WOUT = (ABL & 8192) != 0 ? NB - (NB_REM != 0 ? 1 : 0) : 0;  // ablation: W DMAs left in flight
  for (int sl = 0; sl < nsl; ++sl) {
    const int s = s0 + sl;
    const bool last = sl + 1 == nsl;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int t = 3 * sl + kw;
      if constexpr (PS) {
        // kw 2: W(t) landed (the next strip, issued after it at kw 1, may still fly); else all
        if (kw == 2) {
          if (RESPF && last) {  // the residual loads issued at kw 1 may still fly
            if (a.res && nsplit == 1)
              asm volatile("s_waitcnt vmcnt(%0)" ::"n"(TM * TN) : "memory");
            else
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          } else if (NS_REM == 0 || wave < NS_REM)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS + WOUT) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS - 1 + WOUT) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WOUT) : "memory");
        }
        __builtin_amdgcn_s_barrier();
        const int wnext = kw < 2 ? wk0(s, kw + 1) : (last ? wk0(s, 2) : wk0(s + 1, 0));
        unsigned char* const wdst = WB + ((t + 1) & 1) * W_BYTES;
        if constexpr (!SPREAD) {
          load_w(wnext, wdst);
          if (kw == 1) {
            if (RESPF && last) {  // the residual tile (the last MFMAs hide its latency)
              if (a.res && nsplit == 1) r3t_res_load<TM, TN>(a, rvp, m0 + wave * WM, n0, lane);
            } else {
              load_strip(last ? s : s + 1, smem);  // every wave has split strip s
            }
          }
        }
        if (kw == 0) presplit(smem);
        compute(smem, WB + (t & 1) * W_BYTES, kw, [&](int ni) {
          if constexpr (SPREAD) spread_issue(ni, kw == 1, wnext, wdst, last ? s : s + 1, smem);
        });
        continue;
      }
      if (kw == 1) {
        if (NS_REM == 0 || wave < NS_REM)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS + WOUT) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS - 1 + WOUT) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WOUT) : "memory");
      }
      __builtin_amdgcn_s_barrier();  // W(t) (and the strip) landed for every wave; W(t-1) no longer read
      const int wnext = kw < 2 ? wk0(s, kw + 1) : (last ? wk0(s, 2) : wk0(s + 1, 0));
      unsigned char* const wdst = WB + ((t + 1) & 1) * W_BYTES;
      unsigned char* const sdst = smem + ((sl + 1) & 1) * S_BYTES;
      if constexpr (!SPREAD) {
        load_w(wnext, wdst);
        if (kw == 0) load_strip(last ? s : s + 1, sdst);
      }
      compute(smem + (sl & 1) * S_BYTES, WB + (t & 1) * W_BYTES, kw, [&](int ni) {
        if constexpr (SPREAD) spread_issue(ni, kw == 0, wnext, wdst, last ? s : s + 1, sdst);
      });
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (nsplit > 1 && (ABL & 2) != 0 && a.tile_cnt) {  // in-kernel split-K (conv_r3_kernel.h)
    r3t_splitk_combine<TM, TN, NT>(a, acc, smem, lbid, kz, nsplit, m0 + wave * WM, m0, n0, lane, ainv);
    return;
  }
  if (nsplit > 1 && (ABL & 2) != 0) {  // split-K partials, transposed form: float4 per lane
    float* part = a.part + (size_t)kz * M * a.N;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int m = m0 + wave * WM + mi * 16 + c16, n = n0 + ni * 16 + 4 * gq;
        const x6_f32x4 cs = *reinterpret_cast<const x6_f32x4*>(a.winv + n);
        x6_f32x4 val;
#pragma unroll
        for (int v = 0; v < 4; ++v) val[v] = acc[mi][ni][v] * ainv[mi] * cs[v];
        if (m < M) *reinterpret_cast<x6_f32x4*>(part + (size_t)m * a.N + n) = val;
      }
    return;
  }
  if (nsplit > 1) {  // split-K: this slice's partial sums, scaled back (the reduce adds the rest)
    float* part = a.part + (size_t)kz * M * a.N;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int row = mi * 16 + 4 * gq + v, col = ni * 16 + c16;
          const float si = __shfl(ainv[mi], row & 15, 64);
          const int m = m0 + wave * WM + row, n = n0 + col;
          if (m < M) part[(size_t)m * a.N + n] = acc[mi][ni][v] * si * a.winv[n];
        }
    return;
  }
  if constexpr ((ABL & 32) != 0) {  // ablation: no epilogue (accumulators kept live)
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) asm volatile("" ::"v"(acc[mi][ni]));
    return;
  }
  __syncthreads();
  if constexpr ((ABL & 2) != 0 && EPI == EPI_STD)
    r3t_epilogue_std<TM, TN, NT, false, RESPF, ((ABL >> 8) & 3) | ((ABL >> 9) & 4), STG>(a, acc, smem, m0 + wave * WM, m0, n0, lane, ainv,
                                                                    rvp);
  else
    h3_epilogue16<BM, BN, WM, BN, TM, TN, NT, EPI, false>(a, acc, smem, m0, n0, nt, wave, 0, tid, ainv);
}

template <int BM, int BN, int WM, int EPI, int OCC, int ABL = 0>
inline int launch_conv_h3s_cfg(const ConvArgs& a, hipStream_t st) {
  const ConvSeg& g = a.seg[0];
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  if (!a.wh || !a.winv || a.nseg != 1 || g.KH != 3 || g.KW != 3 || g.stride != 1 || g.pad != 1 || g.C < 32 ||
      (g.C & 31) != 0 || a.Kpad != 9 * g.C || a.OH != g.H || a.OW != g.W || a.N % BN != 0) {
    set_error("conv_h3s: not a one-segment 3x3/s1/p1 conv with C %% 32 == 0 (C=%d Kpad=%d N=%d)", g.C, a.Kpad,
              a.N);
    return SFA_E_UNSUPPORTED;
  }
  if (ks > 1 && (EPI != EPI_STD || (3 * (g.C >> 5)) % ks != 0 || !a.part ||
                 (size_t)ks * a.M * a.N > a.part_floats || a.N % 4 != 0)) {
    set_error("conv_h3s: split-K %d unsupported here (C=%d N=%d)", ks, g.C, a.N);
    return SFA_E_UNSUPPORTED;
  }
  if (2ull * a.N * a.Kpad * 2ull >= (1ull << 31)) {
    set_error("conv_h3s: split weights >= 2 GiB");
    return SFA_E_UNSUPPORTED;
  }
  const long long nblocks = (long long)ceil_div(a.M, BM) * (a.N / BN) * ks;
  if (nblocks <= 0 || nblocks > 0x7fffffffll) {
    set_error("conv_h3s: bad grid (M=%d N=%d)", a.M, a.N);
    return SFA_E_INVALID;
  }
  hipLaunchKernelGGL((conv_h3s_kernel<BM, BN, WM, EPI, OCC, ABL>), dim3((unsigned)nblocks), dim3((BM / WM) * 64), 0,
                     st, a);
  SFA_LAUNCH_CHECK();
  if (ks > 1 && !((ABL & 2) != 0 && a.tile_cnt)) {  // no in-kernel combine: the reduce launch
    const long long nel = (long long)a.M * a.N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((nel + 1023) / 1024)), dim3(256), 0, st, a);
    SFA_LAUNCH_CHECK();
  }
  return SFA_OK;
}

}  // namespace sfa
