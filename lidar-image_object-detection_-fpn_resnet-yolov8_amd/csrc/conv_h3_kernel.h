// Implicit-GEMM convolution, fp16x3 arithmetic, streamlined for gfx950 (CDNA4).
//
// Same GEMM view, operand split and epilogues as conv_x6g_kernel<..., PREC = 1>
// (conv_x6_kernel.h): C[M][N] = A[M][K] * W[N][K]^T over NHWC, A (f32) gathered with
// LDS-DMA and split into two fp16 terms (x s = hi + lo, s the frame's power-of-two
// scale) when a wave reads its fragment, W pre-split on the host into two fp16 terms,
// products hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_f16 with f32 accumulation.
// What differs is the register and instruction budget around the MFMAs:
//  * every wave owns a FIXED set of DMA slots per K-tile (NA A-row groups, NB W-row
//    groups), so the per-row gather origins are NA (not NA + NB) registers and the W
//    source offsets are precomputed (one add per tile);
//  * the gather origin of a row is two registers per segment (pixel index; ih, iw packed
//    as two int16), and the segment count is a template parameter (no dead copies);
//  * the W fragments are read one column block ahead of the MFMAs that use them, and the
//    A fragments of the next k-step are read and split between the current step's MFMAs;
//  * NSTAGE-deep ring (prefetch distance NSTAGE - 1 tiles) and optional N-major tile order
//    (all M-tiles of one weight column block on one XCD: weights larger than an XCD's L2).
// LDS images (16-B quad/chunk q of row R stored at q ^ swz(R); conflict-free ds_read_b128):
//   A rows BK f32:  BK 32 -> 128 B, swz (R >> 1) & 7;  BK 16 -> 64 B, swz (R >> 2) & 3
//   W rows BK fp16: BK 32 ->  64 B, swz (R >> 2) & 3;  BK 16 -> 32 B, swz (R >> 3) & 1
#pragma once

#include "conv_x6_kernel.h"

namespace sfa {

typedef float f32x4_t __attribute__((ext_vector_type(4)));


// Epilogue of the 16x16x32 form (accumulator layout of v_mfma_f32_16x16x32_f16: lane l,
// register v -> row 4 (l >> 4) + v, column l & 15 of its 16x16 tile).  Same semantics as
// x6_epilogue<..., PREC = 1>: scale back by 1/s of the row's frame and winv[n], bias,
// residual, ReLU, store, per-frame max |y|; EPI_HEAD stages ReLU(conv3x3 + b) of each head
// in LDS and applies its 1x1 conv, channel-planar out.
template <int BM, int BN, int WM, int WN, int TM, int TN, int NT, int EPI, bool RES_UP = true>
__device__ __forceinline__ void h3_epilogue16(const ConvArgs& a, f32x4_t (&acc)[TM][TN], unsigned char* smem,
                                              int m0, int n0, int nt, int wave, int wn, int tid,
                                              const float (&ainv)[TM]) {
  // wave = the wave's row-block index (wm), wn its column-block index (WN columns each)
  const int M = a.M, lane = tid & 63, c16 = lane & 15, g = lane >> 4;
  float rinv[TM][4];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int v = 0; v < 4; ++v) rinv[mi][v] = __shfl(ainv[mi], 4 * g + v, 64);
  if constexpr (EPI == EPI_STD) {
    AmaxRows am(a.OH * a.OW, m0);
    float rv[TM][TN][4];  // residual tile loaded up front
    if (a.res) {
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int m = min(m0 + wave * WM + mi * 16 + 4 * g + v, M - 1);
            rv[mi][ni][v] = a.res[(size_t)m * a.N + n0 + wn * WN + ni * 16 + c16];
          }
    }
    if (RES_UP && a.res_up) {
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int m = min(m0 + wave * WM + mi * 16 + 4 * g + v, M - 1);
            rv[mi][ni][v] = res_up_sample(a, m, n0 + wn * WN + ni * 16 + c16);
          }
    }
    // the columns' bias / winv all loaded before the first store (round 5: per column block they sat
    // behind the previous block's stores, which may alias them for hipcc: one round trip each)
    float bng[TN], csg[TN];
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int n = n0 + wn * WN + ni * 16 + c16;
      bng[ni] = a.bias ? a.bias[n] : 0.f;
      csg[ni] = a.winv[n];
    }
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int n = n0 + wn * WN + ni * 16 + c16;
      const float bn = bng[ni];
      const float cs = csg[ni];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int m = m0 + wave * WM + mi * 16 + 4 * g + v;
          if (m < M) {
            float val = acc[mi][ni][v] * rinv[mi][v] * cs + bn;
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
    // All BM rows of one head's ReLU(conv3x3 + b) staged in LDS at once, the block's 1x1
    // weights beside them (staged once, not re-read from global per output); the 1x1 conv
    // then runs LPR lanes per row (KPL of the 64 inputs each, shuffle-reduced): two barriers
    // per head.
    static_assert(BN % 64 == 0, "whole heads per block");
    constexpr int HPB = BN / 64;
    constexpr int LPR = NT / BM, KPL = 64 / LPR;
    static_assert(NT % BM == 0 && LPR >= 1 && LPR <= 8 && (LPR & (LPR - 1)) == 0, "1x1 lanes per row");
    float* T = reinterpret_cast<float*>(smem);  // [BM][65]
    float* WH = T + BM * 65;                    // [HPB][4][64]
    for (int i = tid; i < HPB * 256; i += NT) WH[i] = a.hw1[nt * HPB * 256 + i];
    const int prow = tid / LPR, q = tid % LPR;
    const int pm = m0 + prow;
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
      for (int ni = 0; ni < TN; ++ni) {  // the wave's column blocks that belong to head hh
        const int gi = wn * TN + ni;
        if ((gi >> 2) != hh) continue;
        const int col = (gi - 4 * hh) * 16 + c16;  // column within the head
        const float bn = a.bias[n0 + 64 * hh + col];
        const float cs = a.winv[n0 + 64 * hh + col];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int row = wave * WM + mi * 16 + 4 * g + v;
            T[row * 65 + col] = fmaxf(acc[mi][ni][v] * rinv[mi][v] * cs + bn, 0.f);
          }
      }
      __syncthreads();
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
      const float* tr = T + prow * 65 + q * KPL;
      const float* wq = WH + hh * 256 + q * KPL;
#pragma unroll
      for (int k = 0; k < KPL; ++k) {
        const float t = tr[k];
        s0 = fmaf(t, wq[k], s0);
        s1 = fmaf(t, wq[64 + k], s1);
        s2 = fmaf(t, wq[128 + k], s2);
        s3 = fmaf(t, wq[192 + k], s3);
      }
#pragma unroll
      for (int o = 1; o < LPR; o <<= 1) {
        s0 += __shfl_xor(s0, o, 64);
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
        s3 += __shfl_xor(s3, o, 64);
      }
      if (q == 0 && pm < M) {
        const float* hb = a.hb1 + head * 4;
        float* o = a.hout + (size_t)hoff * M + pm;
        o[0] = s0 + hb[0];
        if (ch > 1) o[(size_t)M] = s1 + hb[1];
        if (ch > 2) o[2 * (size_t)M] = s2 + hb[2];
        if (ch > 3) o[3 * (size_t)M] = s3 + hb[3];
      }
      __syncthreads();
    }
  }
}

// Stem + max-pool (fpn_resnet.py:179-182: conv1 -> bn1 -> relu -> maxpool 3x3/s2/p1) for
// the 32x32x16 form. The block's BM rows are one TRH x 16 tile (th, tw) of frame b of the
// conv output (TRH = BM / 16); ReLU(conv + b) goes to LDS, then the block writes the pooled
// cells whose window touches the tile: pooled rows TR th .. TR th + TR (TR = TRH / 2),
// columns 8 tw .. 8 tw + 8 (window rows 2 py - 1 .. 2 py + 1 cut to the tile). Cells whose
// window lies wholly inside the tile (j in 1..TR-1, i in 1..7) have one writer and are
// stored; the border cells are shared with the up/left neighbours and combined with
// atomicMax on the f32 bits, exact because the values are >= +0 (ReLU, canonical +0) and
// the pooled buffer is zeroed first. The pooled max is the conv output's max, recorded per
// frame as the stem's amax (maxpool keeps it).
template <int BM, int BN, int WM, int TM, int TN, int NT>
__device__ __forceinline__ void h3_pool_epilogue(const ConvArgs& a, x6_f32x16 (&acc)[TM][TN],
                                                 unsigned char* smem, int m0, int wave, int tid,
                                                 const float (&ainv)[TM]) {
  constexpr int LD = BN + 4;  // float4-aligned rows
  float* T = reinterpret_cast<float*>(smem);
  const int lane = tid & 63, r = lane & 31, h = lane >> 5;
  float mx = 0.f;
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) {
    const int n = ni * 32 + r;
    const float bn = a.bias[n];
    const float cs = a.winv[n];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = wave * WM + mi * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        const float rinv = __shfl(ainv[mi], (v & 3) + 8 * (v >> 2) + 4 * h, 64);
        float val = acc[mi][ni][v] * rinv * cs + bn;
        val = val > 0.f ? val : 0.f;
        T[row * LD + n] = val;
        mx = fmaxf(mx, val);
      }
  }
  const int P = a.OH * a.OW;
  const int b = m0 / P;
  if (a.amax_out)
    amax_commit_block<NT / 64>(a.amax_out, b, mx, 0.f, T + BM * LD);  // includes __syncthreads
  else
    __syncthreads();
  constexpr int TRH = BM / 16, TR = TRH / 2;  // conv rows / pooled rows per tile
  const int tile = (m0 - b * P) / BM, tw_n = a.OW >> 4;
  const int th = tile / tw_n, tw = tile - th * tw_n;
  const int PH = a.OH >> 1, PW = a.OW >> 1;
  constexpr int C4 = BN / 4;
  for (int idx = tid; idx < (TR + 1) * 9 * C4; idx += NT) {
    const int c4 = idx % C4, cell = idx / C4;
    const int j = cell / 9, i = cell - 9 * (cell / 9);
    const int py = TR * th + j, px = 8 * tw + i;
    if (py >= PH || px >= PW) continue;
    const int r0 = 2 * j - 1 > 0 ? 2 * j - 1 : 0, r1 = 2 * j + 1 < TRH - 1 ? 2 * j + 1 : TRH - 1;
    const int q0 = 2 * i - 1 > 0 ? 2 * i - 1 : 0, q1 = 2 * i + 1 < 15 ? 2 * i + 1 : 15;
    x6_f32x4 m = {0.f, 0.f, 0.f, 0.f};
    for (int rr = r0; rr <= r1; ++rr)
      for (int qq = q0; qq <= q1; ++qq) {
        const x6_f32x4 t = *reinterpret_cast<const x6_f32x4*>(T + (rr * 16 + qq) * LD + 4 * c4);
#pragma unroll
        for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], t[e]);
      }
    float* dst = a.y + ((size_t)(b * PH + py) * PW + px) * BN + 4 * c4;
    if (j >= 1 && j < TR && i >= 1 && i <= 7) {
      *reinterpret_cast<x6_f32x4*>(dst) = m;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (m[e] > 0.f) atomicMax(reinterpret_cast<unsigned*>(dst) + e, __float_as_uint(m[e]));
    }
  }
}

// ABL (variants for tools/convbench): 1 = no DMA in the K loop (ablation), 2 = software-
// pipelined fragment reads (compute_pipe), 4 = s_setprio 1 for the second half of the waves.
// MF: 0 = v_mfma_f32_32x32x16_f16 (32-row / 32-column wave sub-tiles), 1 = v_mfma_f32_16x16x32_f16
// (16 x 16 sub-tiles, BK 32: same LDS reads and registers per MAC; the chip holds a higher
// clock under the 16x16 shape on random data, MI355X_MICROARCH.md 'DVFS give-back' (7)).
// WN (16x16x32 form only): columns per wave; WN < BN lays the waves out 2-D, (BM / WM) along M
// times (BN / WN) along N, so each wave reads WN columns of W fragments instead of all BN
// (fewer LDS bytes per MAC) and splits its WM rows of A.
// RU: the epilogue handles an upsampled residual (a.res_up); instances without it (every conv but the
// FPN skip convs) keep the residual tile in registers without spilling.
// In-kernel split-K combine (round 5; conv_h3s_kernel, whose partials are float4 rows, replaces
// splitk_reduce_kernel with it when the conv has a ticket array, ConvArgs::tile_cnt — conv_h3_kernel's
// element-strided partials made write-through cost 30-38 us per layer4 conv, profiles/r05c_*, so it
// keeps the reduce launch): every slice stores its partial tile write-through (sc1), waits for the stores
// (s_waitcnt vmcnt(0)) in every wave, and after a workgroup barrier one lane takes a ticket for the
// output tile with an agent-scope atomic add; the slice whose add returns nsplit - 1 is the last to
// finish and, after a second barrier, reads the other slices' partials with sc1 loads and applies the
// reduce kernel's epilogue (slices added in slice order 0 .. nsplit-1 with its own partial from
// registers, + bias, + residual, ReLU, per-frame max): bit-identical to the reduce launch.  This is
// the producer / consumer hand-off of MI355X_MICROARCH.md (inter-workgroup visibility: sc1 stores,
// drained, one atomic add per storing workgroup, the last adder reads with sc1 loads); the tickets are
// zeroed with the forward's amax words.  `flag` is an LDS word no wave uses meanwhile.
__device__ __forceinline__ bool splitk_ticket(unsigned* cnt, int tile, int nsplit, unsigned* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores have completed
  __syncthreads();                                   // ... and every other wave's
  if (threadIdx.x == 0) *flag = __hip_atomic_fetch_add(cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return *flag == (unsigned)(nsplit - 1);
}

template <int BM, int BN, int WM, int EPI, int OCC, int BK, int NSTAGE, int NSEG, bool NMAJ = false,
          int ABL = 0, int MF = 0, int WN = BN, bool RU = false>
__global__ void __launch_bounds__((BM / WM) * (BN / WN) * 64, OCC) conv_h3_kernel(const ConvArgs a) {
  static_assert(BK == 16 || BK == 32, "BK");
  static_assert(NSTAGE >= 2 && NSTAGE <= 4, "ring depth");
  static_assert(NSEG == 1 || NSEG == 2, "segments");
  static_assert(MF == 0 || (BK == 32 && WM % 16 == 0), "16x16x32 form: BK 32");
  static_assert(WN == BN || (MF == 1 && BN % WN == 0 && WN % 16 == 0), "2-D wave layout: 16x16x32 form");
  constexpr int NWM = BM / WM, NW = NWM * (BN / WN), NT = NW * 64;
  constexpr int MT = MF ? 16 : 32;  // MFMA sub-tile edge
  constexpr int TM = WM / MT, TN = WN / MT;
  constexpr int KST = BK / 16;
  constexpr int AROW = BK * 4, BROW = BK * 2;  // bytes per LDS row
  constexpr int A_BYTES = BM * AROW, TERM_B = BN * BROW;
  constexpr int STAGE = A_BYTES + 2 * TERM_B;
  constexpr int A_RPD = 1024 / AROW, B_RPD = 1024 / BROW;  // rows per DMA instruction
  constexpr int ND_A = BM / A_RPD, ND_BT = BN / B_RPD, ND_B = 2 * ND_BT;
  static_assert(BM % A_RPD == 0 && BN % B_RPD == 0 && BN % 32 == 0 && WM % 32 == 0, "tile");
  static_assert(ND_A % NW == 0, "A DMA groups per wave");
  constexpr int NA = ND_A / NW;
  constexpr int NB = (ND_B + NW - 1) / NW;
  constexpr int NB_REM = ND_B % NW;  // if != 0: waves < NB_REM issue NB W DMAs, the rest NB - 1
  constexpr int HCH = BM < 128 ? BM : 128;
  constexpr int HEAD_BYTES = EPI != EPI_HEAD ? 0 : MF == 1 ? BM * 65 * 4 + (BN / 64) * 1024 : HCH * 65 * 4;
  constexpr int POOL_BYTES = EPI == EPI_POOL ? BM * (BN + 4) * 4 + 2 * NW * 4 : 0;
  constexpr int LDS_A = NSTAGE * STAGE > HEAD_BYTES ? NSTAGE * STAGE : HEAD_BYTES;
  constexpr int LDS_BYTES = LDS_A > POOL_BYTES ? LDS_A : POOL_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  static_assert(EPI != EPI_POOL || ((BM == 128 || BM == 256) && MF == 0), "pool epilogue: (BM/16)x16 tiles");

  // 16x16x32 reads: lane l takes row l & 15, quads / chunk by l >> 4; the extra XOR terms
  // make the ds_read_b128 lane groups {0-3,12-15,20-27}, ... hit 16 distinct bank quads
  auto swzA = [](int R) {
    return MF ? (((R >> 1) & 7) ^ (((R & 15) + 4) >> 2 & 2)) : (BK == 16 ? ((R >> 2) & 3) : ((R >> 1) & 7));
  };
  auto swzB = [](int R) {
    return MF ? (((R >> 2) & 3) ^ ((((R & 15) + 4) >> 3) & 1)) : (BK == 16 ? ((R >> 3) & 1) : ((R >> 2) & 3));
  };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % NWM, wn = wave / NWM;  // the wave's row / column block
  const int n_tiles = a.N / BN;
  const int m_tiles = (a.M + BM - 1) / BM;
  const int nsplit = a.ksplit > 1 ? a.ksplit : 1;
  int lbid = xcd_remap(blockIdx.x, gridDim.x);
  const int kz = lbid / (m_tiles * n_tiles);  // split-K slice of this block
  lbid -= kz * (m_tiles * n_tiles);
  int mt, nt;
  if constexpr (NMAJ) {
    nt = lbid / m_tiles;
    mt = lbid - nt * m_tiles;
  } else {
    mt = lbid / n_tiles;
    nt = lbid - mt * n_tiles;
  }
  const int m0 = mt * BM, n0 = nt * BN;
  const int M = a.M;

  // ---- A DMA slots: groups d = wave + NW * i, rows A_RPD * d + lane / QPR ----
  constexpr int QPR = AROW / 16;
  const int arow_in = lane / QPR;
  // the lane's logical f32 quad: every slot's row has the same swizzle (BK 16: A_RPD = 16;
  // BK 32: rows 8d + lane/8 with d of the wave's parity, NW even)
  static_assert(BK == 16 || NW % 2 == 0, "swizzle period");
  const int kq = (lane % QPR) ^ swzA(A_RPD * wave + arow_in);
  int r_pix[NSEG][NA], r_ihw[NSEG][NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = m0 + A_RPD * (wave + NW * i) + arow_in;
    const bool ok = m < M;
    const int mm = ok ? m : 0;
    int ow, oh, b;
    if constexpr (EPI == EPI_POOL) {  // block = one (BM/16)x16 tile of a frame, raster order
      const int P = a.OH * a.OW;
      b = mm / P;
      const int rem = mm - b * P, tile = rem / BM, loc = rem % BM, tw_n = a.OW >> 4;
      const int th = tile / tw_n;
      oh = th * (BM / 16) + (loc >> 4);
      ow = ((tile - th * tw_n) << 4) + (loc & 15);
    } else {
      const int t = fast_div(mm, a.fd_ow);  // round 5: multiply-high divisions (a.fd_ow / fd_oh)
      ow = mm - t * a.OW;
      b = fast_div(t, a.fd_oh);
      oh = t - b * a.OH;
    }
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
      const ConvSeg& g = a.seg[sg];
      const int ih = ok ? oh * g.stride - g.pad : -16384;
      const int iw = ow * g.stride - g.pad;
      r_pix[sg][i] = (b * g.H + ih) * g.W + iw;
      r_ihw[sg][i] = (ih << 16) | (iw & 0xffff);
    }
  }
  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.seg[0].x), (short)0, (int)a.seg[0].bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.seg[NSEG - 1].x), (short)0, (int)a.seg[NSEG - 1].bytes, 0x00020000);

  // ---- W DMA slots: groups e = wave + NW * j (term e / ND_BT, rows (e % ND_BT) * B_RPD + ..) ----
  const int wst = a.wstride ? a.wstride : a.Kpad;  // row stride of the fp16 terms
  const unsigned term_bytes = (unsigned)a.N * (unsigned)wst * 2u;
  const __amdgpu_buffer_rsrc_t rsw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.wh), (short)0, (int)(2 * term_bytes), 0x00020000);
  constexpr int CPR = BROW / 16;
  int boff[NB];  // int array + unsigned cast at the use: other forms make hipcc's host pass drop the kernel stub
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int e = wave + NW * j < ND_B ? wave + NW * j : ND_B - 1;
    const int t = e / ND_BT;
    const int R = (e % ND_BT) * B_RPD + lane / CPR;
    const int lc = (lane % CPR) ^ swzB(R);
    boff[j] = (int)(t * term_bytes) + (int)(((n0 + R) * wst + a.wk0 + 8 * lc) << 1);
  }

  // fp16x3 scale of the frame of this lane's A row in each 32-row MFMA tile: the block's first two
  // frames' scales by uniform loads, rows of later frames (small maps) their own
  float as[TM], ainv[TM];
  {
    const int P = a.OH * a.OW, f0 = m0 / P, fb = (f0 + 1) * P;
    float sA, iA, sB, iB;
    amax_frame_scale2(a.amax_in, NSEG, f0, min(f0 + 1, (M - 1) / P), sA, iA, sB, iB);
    if (fb >= M) {
      sB = sA;
      iB = iA;
    }
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = min(m0 + wm * WM + mi * MT + (lane & (MT - 1)), M - 1);
      if (m < fb) {
        as[mi] = sA;
        ainv[mi] = iA;
      } else if (m < fb + P) {
        as[mi] = sB;
        ainv[mi] = iB;
      } else {
        as[mi] = amax_frame_scale(a.amax_in, NSEG, m / P, ainv[mi]);
      }
    }
  }

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
    for (int i = 0; i < NA; ++i) {
      const int ih = r_ihw[SG][i] >> 16;
      const int iw = (int)(short)(r_ihw[SG][i] & 0xffff);
      const bool ok = tap_ok & ((unsigned)(ih + kh) < (unsigned)g.H) & ((unsigned)(iw + kw) < (unsigned)g.W);
      const unsigned off = ok ? (unsigned)((((r_pix[SG][i] + toff) << g.logC) + c) << 2) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(S + (wave + NW * i) * 1024), 16, off, 0, 0, 0);
    }
  };
  auto load_tile = [&](int kt, unsigned char* S) {
    const int k0 = kt * BK;
    if constexpr (NSEG == 2) {
      if (k0 >= a.kseg1)
        load_a(std::integral_constant<int, 1>(), rs1, k0 - a.kseg1, S);
      else
        load_a(std::integral_constant<int, 0>(), rs0, k0, S);
    } else {
      load_a(std::integral_constant<int, 0>(), rs0, k0, S);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (NB_REM == 0 || j < NB - 1 || wave < NB_REM)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsw, (__attribute__((address_space(3))) void*)(S + A_BYTES + (wave + NW * j) * 1024), 16,
            (unsigned)(boff[j] + 2 * k0), 0, 0, 0);
    }
  };

  typedef typename std::conditional<MF == 1, f32x4_t, x6_f32x16>::type acc_t;
  acc_t acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int v = 0; v < (MF ? 4 : 16); ++v) acc[mi][ni][v] = 0.f;

  const int r = lane & 31, h = lane >> 5;
  // per-lane LDS byte offsets (stage-relative)
  int aoff[TM][2 * KST];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    const int R = wave * WM + mi * 32 + r;
#pragma unroll
    for (int q = 0; q < 2 * KST; ++q) aoff[mi][q] = R * AROW + ((((q >> 1) * 4 + 2 * h + (q & 1)) ^ swzA(R)) << 4);
  }
  int bbase[KST];
#pragma unroll
  for (int s = 0; s < KST; ++s) bbase[s] = A_BYTES + r * BROW + (((2 * s + h) ^ swzB(r)) << 4);

  auto read_a = [&](const unsigned char* S, int s, f16x8_t (&hf)[2][TM]) {
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const x6_f32x4 q0 = *reinterpret_cast<const x6_f32x4*>(S + aoff[mi][2 * s]);
      const x6_f32x4 q1 = *reinterpret_cast<const x6_f32x4*>(S + aoff[mi][2 * s + 1]);
      f16x4_t t0, t1, u0, u1;
      split2h(q0, as[mi], t0, t1);
      split2h(q1, as[mi], u0, u1);
      hf[0][mi] = __builtin_shufflevector(t0, u0, 0, 1, 2, 3, 4, 5, 6, 7);
      hf[1][mi] = __builtin_shufflevector(t1, u1, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  };
  auto compute = [&](const unsigned char* S) {
    if constexpr (MF == 0) {
#pragma unroll
    for (int s = 0; s < KST; ++s) {
      f16x8_t hf[2][TM];
      read_a(S, s, hf);
      const unsigned char* SB = S + bbase[s];
      f16x8_t b0 = *reinterpret_cast<const f16x8_t*>(SB);
      f16x8_t b1 = *reinterpret_cast<const f16x8_t*>(SB + TERM_B);
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        f16x8_t c0 = b0, c1 = b1;
        if (ni + 1 < TN) {  // next column block's fragments, one block ahead of their MFMAs
          b0 = *reinterpret_cast<const f16x8_t*>(SB + (ni + 1) * 32 * BROW);
          b1 = *reinterpret_cast<const f16x8_t*>(SB + TERM_B + (ni + 1) * 32 * BROW);
        }
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          x6_f32x16 cc = acc[mi][ni];
          cc = __builtin_amdgcn_mfma_f32_32x32x16_f16(hf[1][mi], c0, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_32x32x16_f16(hf[0][mi], c1, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_32x32x16_f16(hf[0][mi], c0, cc, 0, 0, 0);
          acc[mi][ni] = cc;
        }
      }
    }
    }
  };

  // Software-pipelined form (ABL & 2): the scheduler may not move instructions across
  // the column-block boundaries, so the W fragments are read two column blocks ahead
  // (across the k-step boundary too) and the next k-step's A quads are read after the
  // first column block and split after the third, between MFMAs.
  auto compute_pipe = [&](const unsigned char* S) {
    if constexpr (MF == 0) {
    constexpr int NSTEP = KST * TN;  // (k-step, column block) pairs in program order
    f16x8_t bq[3][2];                // W fragment ring: pair p lives in slot p % 3
    x6_f32x4 qa[TM][2];
    f16x8_t hf[2][TM], hn[2][TM];
    auto read_b = [&](int p) {
      const int s = p / TN, ni = p % TN;
      const unsigned char* SB = S + bbase[s] + ni * 32 * BROW;
      bq[p % 3][0] = *reinterpret_cast<const f16x8_t*>(SB);
      bq[p % 3][1] = *reinterpret_cast<const f16x8_t*>(SB + TERM_B);
    };
    auto read_qa = [&](int s) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        qa[mi][0] = *reinterpret_cast<const x6_f32x4*>(S + aoff[mi][2 * s]);
        qa[mi][1] = *reinterpret_cast<const x6_f32x4*>(S + aoff[mi][2 * s + 1]);
      }
    };
    auto split_qa = [&](f16x8_t (&dst)[2][TM]) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        f16x4_t t0, t1, u0, u1;
        split2h(qa[mi][0], as[mi], t0, t1);
        split2h(qa[mi][1], as[mi], u0, u1);
        dst[0][mi] = __builtin_shufflevector(t0, u0, 0, 1, 2, 3, 4, 5, 6, 7);
        dst[1][mi] = __builtin_shufflevector(t1, u1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    };
    read_qa(0);
    read_b(0);
    if (NSTEP > 1) read_b(1);
    split_qa(hf);
#pragma unroll
    for (int p = 0; p < NSTEP; ++p) {
      const int s = p / TN, ni = p % TN;
      if (p + 2 < NSTEP) read_b(p + 2);
      if (s + 1 < KST && ni == 0) read_qa(s + 1);
      if (s + 1 < KST && ni == (TN > 2 ? 2 : TN - 1)) split_qa(hn);
      const f16x8_t c0 = bq[p % 3][0], c1 = bq[p % 3][1];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        x6_f32x16 cc = acc[mi][ni];
        cc = __builtin_amdgcn_mfma_f32_32x32x16_f16(hf[1][mi], c0, cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_32x32x16_f16(hf[0][mi], c1, cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_32x32x16_f16(hf[0][mi], c0, cc, 0, 0, 0);
        acc[mi][ni] = cc;
      }
      if (ni == TN - 1 && s + 1 < KST) {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          hf[0][mi] = hn[0][mi];
          hf[1][mi] = hn[1][mi];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    }
  };

  // 16x16x32 form (one k-step per BK 32 tile): W fragments two column blocks ahead, as
  // compute_pipe; lane l reads A row l & 15 quads 2 (l >> 4), +1 and W row l & 15 chunk l >> 4.
  auto compute16 = [&](const unsigned char* S) {
    if constexpr (MF == 1) {
      const int c16 = lane & 15, g = lane >> 4;
      f16x8_t hf[2][TM];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const int R = wm * WM + mi * 16 + c16;
        const x6_f32x4 q0 = *reinterpret_cast<const x6_f32x4*>(S + R * AROW + (((2 * g) ^ swzA(R)) << 4));
        const x6_f32x4 q1 = *reinterpret_cast<const x6_f32x4*>(S + R * AROW + (((2 * g + 1) ^ swzA(R)) << 4));
        f16x4_t t0, t1, u0, u1;
        split2h(q0, as[mi], t0, t1);
        split2h(q1, as[mi], u0, u1);
        hf[0][mi] = __builtin_shufflevector(t0, u0, 0, 1, 2, 3, 4, 5, 6, 7);
        hf[1][mi] = __builtin_shufflevector(t1, u1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      const unsigned char* SB = S + A_BYTES + (wn * WN + c16) * BROW + ((g ^ swzB(c16)) << 4);
      f16x8_t bq[3][2];
      auto read_b = [&](int ni) {
        bq[ni % 3][0] = *reinterpret_cast<const f16x8_t*>(SB + ni * 16 * BROW);
        bq[ni % 3][1] = *reinterpret_cast<const f16x8_t*>(SB + TERM_B + ni * 16 * BROW);
      };
      read_b(0);
      if (TN > 1) read_b(1);
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        if (ni + 2 < TN) read_b(ni + 2);
        const f16x8_t c0 = bq[ni % 3][0], c1 = bq[ni % 3][1];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          f32x4_t cc = acc[mi][ni];
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(hf[1][mi], c0, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(hf[0][mi], c1, cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(hf[0][mi], c0, cc, 0, 0, 0);
          acc[mi][ni] = cc;
        }
        if constexpr ((ABL & 2) != 0) __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  const int nk = a.Kpad / BK / nsplit;  // this block's K-tiles: kt0 .. kt0 + nk - 1
  const int kt0 = kz * nk;
  // ring: tile kt lives in stage kt % NSTAGE; tiles kt+1 .. kt+NSTAGE-1 are in flight
#pragma unroll
  for (int p = 0; p < NSTAGE - 1; ++p) load_tile(kt0 + (p < nk ? p : nk - 1), smem + p * STAGE);
  if constexpr ((ABL & 4) != 0) {
    if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }
  int st_cur = 0, st_next = NSTAGE - 1;
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's DMAs of tile kt have landed (later tiles' may still be in flight)
    constexpr int PER = NA + NB;
    if (NB_REM == 0 || wave < NB_REM)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTAGE - 2) * PER) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTAGE - 2) * (PER - 1)) : "memory");
    __builtin_amdgcn_s_barrier();  // every wave's: stage kt complete; stage kt-1 no longer read
    if constexpr (!(ABL & 1)) {
      const int kn = kt + NSTAGE - 1;
      load_tile(kt0 + (kn < nk ? kn : nk - 1), smem + st_next * STAGE);
    }
    if constexpr (MF == 1)
      compute16(smem + st_cur * STAGE);
    else if constexpr ((ABL & 2) != 0)
      compute_pipe(smem + st_cur * STAGE);
    else
      compute(smem + st_cur * STAGE);
    st_cur = st_cur + 1 == NSTAGE ? 0 : st_cur + 1;
    st_next = st_next + 1 == NSTAGE ? 0 : st_next + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (nsplit > 1) {  // split-K: this slice's partial sums, scaled back (the reduce adds the rest)
    float* part = a.part + (size_t)kz * M * a.N;
    // the columns' winv loaded before the first partial store (they may alias for hipcc: round 5)
    float wvg[TN];
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) wvg[ni] = a.winv[n0 + wn * WN + ni * (MF ? 16 : 32) + (MF ? (lane & 15) : (lane & 31))];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int v = 0; v < (MF ? 4 : 16); ++v) {
          int row, col;
          if constexpr (MF == 1) {
            row = mi * 16 + 4 * (lane >> 4) + v;
            col = ni * 16 + (lane & 15);
          } else {
            row = mi * 32 + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
            col = ni * 32 + (lane & 31);
          }
          const float si = __shfl(ainv[mi], MF ? (row & 15) : (row & 31), 64);
          const int m = m0 + wm * WM + row, n = n0 + wn * WN + col;
          if (m < M) part[(size_t)m * a.N + n] = acc[mi][ni][v] * si * wvg[ni];
        }
    return;
  }
  __syncthreads();
  if constexpr (EPI == EPI_POOL)
    h3_pool_epilogue<BM, BN, WM, TM, TN, NT>(a, acc, smem, m0, wave, tid, ainv);
  else if constexpr (MF == 1)
    h3_epilogue16<BM, BN, WM, WN, TM, TN, NT, EPI, RU>(a, acc, smem, m0, n0, nt, wm, wn, tid, ainv);
  else
    x6_epilogue<BM, BN, WM, BN, TM, TN, NT, EPI, 1, RU>(a, acc, smem, m0, n0, nt, wave, 0, tid, ainv);
}

// Split-K reduce: y = sum_z part[z] + bias (+ residual) (ReLU), per-frame max |y| — the
// EPI_STD epilogue over float4 column groups; the slices are added in a fixed order.
static __global__ void __launch_bounds__(256) splitk_reduce_kernel(const ConvArgs a) {
  const int M = a.M, N = a.N;
  const long long e0 = (long long)blockIdx.x * 1024;
  const long long e = e0 + 4 * threadIdx.x;
  AmaxRows am(a.OH * a.OW, (int)(e0 / N));
  if (e < (long long)M * N) {
    const int m = (int)(e / N), n = (int)(e - (long long)m * N);
    x6_f32x4 s = *reinterpret_cast<const x6_f32x4*>(a.part + e);
    for (int z = 1; z < a.ksplit; ++z) s += *reinterpret_cast<const x6_f32x4*>(a.part + (size_t)z * M * N + e);
    s += *reinterpret_cast<const x6_f32x4*>(a.bias + n);
    if (a.res) s += *reinterpret_cast<const x6_f32x4*>(a.res + e);
    if (a.relu) {
#pragma unroll
      for (int i = 0; i < 4; ++i) s[i] = fmaxf(s[i], 0.f);
    }
    *reinterpret_cast<x6_f32x4*>(a.y + e) = s;
    if (a.amax_out) am.add(a.amax_out, m, fmaxf(fmaxf(fabsf(s[0]), fabsf(s[1])), fmaxf(fabsf(s[2]), fabsf(s[3]))));
  }
  if (a.amax_out) {
    __shared__ float red[8];
    amax_commit_block<4>(a.amax_out, am.fb0, am.mx0, am.mx1, red);
  }
}

template <int BM, int BN, int WM, int EPI, int OCC, int BK, int NSTAGE, bool NMAJ = false, int ABL = 0,
          int MF = 0, int WN = BN>
inline int launch_conv_h3_cfg(const ConvArgs& a, hipStream_t st) {
  if (!a.wh || !a.winv || a.Kpad % BK != 0 || (a.nseg == 2 && a.kseg1 % BK != 0) || a.N % BN != 0) {
    set_error("conv_h3: K/N not aligned to the tile or no split weights (Kpad=%d kseg1=%d N=%d)", a.Kpad,
              a.kseg1, a.N);
    return SFA_E_UNSUPPORTED;
  }
  if (a.wstride && (a.wstride < a.wk0 + a.Kpad || a.wk0 % 8 != 0)) {
    set_error("conv_h3: K slice [%d, %d) outside the weight rows (stride %d)", a.wk0, a.wk0 + a.Kpad, a.wstride);
    return SFA_E_INVALID;
  }
  if (2ull * a.N * (a.wstride ? a.wstride : a.Kpad) * 2ull >= (1ull << 31)) {
    set_error("conv_h3: split weights >= 2 GiB");
    return SFA_E_UNSUPPORTED;
  }
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  if (ks > 1 && (EPI != EPI_STD || (a.Kpad / BK) % ks != 0 || !a.part ||
                 (size_t)ks * a.M * a.N > a.part_floats || a.N % 4 != 0)) {
    set_error("conv_h3: split-K %d unsupported here (Kpad=%d N=%d)", ks, a.Kpad, a.N);
    return SFA_E_UNSUPPORTED;
  }
  const long long nblocks = (long long)ceil_div(a.M, BM) * (a.N / BN) * ks;
  if (nblocks <= 0 || nblocks > 0x7fffffffll) {
    set_error("conv_h3: bad grid (M=%d N=%d)", a.M, a.N);
    return SFA_E_INVALID;
  }
  ConvArgs c = a;  // the row decomposition's multiply-high divisions
  c.fd_ow = make_fast_div((unsigned)a.OW);
  c.fd_oh = make_fast_div((unsigned)a.OH);
  if (a.res_up) {  // FPN skip convs (one segment): the instance with the upsampled-residual epilogue
    if (a.nseg != 1) {
      set_error("conv_h3: upsampled residual with two K-segments");
      return SFA_E_UNSUPPORTED;
    }
    hipLaunchKernelGGL((conv_h3_kernel<BM, BN, WM, EPI, OCC, BK, NSTAGE, 1, NMAJ, ABL, MF, WN, true>),
                       dim3((unsigned)nblocks), dim3((BM / WM) * (BN / WN) * 64), 0, st, c);
  } else if (a.nseg == 2) {
    hipLaunchKernelGGL((conv_h3_kernel<BM, BN, WM, EPI, OCC, BK, NSTAGE, 2, NMAJ, ABL, MF, WN>),
                       dim3((unsigned)nblocks), dim3((BM / WM) * (BN / WN) * 64), 0, st, c);
  } else {
    hipLaunchKernelGGL((conv_h3_kernel<BM, BN, WM, EPI, OCC, BK, NSTAGE, 1, NMAJ, ABL, MF, WN>),
                       dim3((unsigned)nblocks), dim3((BM / WM) * (BN / WN) * 64), 0, st, c);
  }
  SFA_LAUNCH_CHECK();
  if (ks > 1) {  // the slices' partials combined by the reduce launch (element-strided partials: no tickets)
    const long long nel = (long long)a.M * a.N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((nel + 1023) / 1024)), dim3(256), 0, st, a);
    SFA_LAUNCH_CHECK();
  }
  return SFA_OK;
}

}  // namespace sfa
