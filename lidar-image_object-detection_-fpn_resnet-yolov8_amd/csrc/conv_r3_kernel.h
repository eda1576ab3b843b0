// Implicit-GEMM convolution, fp16x3 arithmetic, A operand in REGISTERS (gfx950 / CDNA4).
//
// Same GEMM view, operand split, scales and epilogues as conv_h3_kernel<..., MF = 1>
// (conv_h3_kernel.h): C[M][N] = A[M][K] * W[N][K]^T over NHWC, products hi*hi + hi*lo + lo*hi
// on v_mfma_f32_16x16x32_f16 with f32 accumulation, BK = 32 (one MFMA k-step per K-tile).
// What differs is where A lives. The waves are stacked along M (each wave owns WM rows x all
// BN columns), so no wave ever reads another wave's A rows: each lane loads its own fragment
// (row l & 15 of each 16-row sub-tile, f32 k = 8 (l >> 4) .. +7 = 32 contiguous bytes of one
// input pixel) straight into VGPRs with two buffer loads, one K-tile ahead, and splits it
// into the fp16 terms at the top of the K-tile. Only the weights (shared by all waves) go
// through LDS, by LDS-DMA into an NSTAGE-deep ring. Compared with staging A through LDS:
//  * the per-tile A DMA pieces, their LDS writes and the A fragment ds_reads are gone;
//  * after a K-tile's barrier a wave has nothing to wait for: its A fragment arrived during
//    the previous tile and (NSTAGE 3) the first two W fragment blocks were read before the
//    barrier, so the MFMAs restart at once instead of behind DMA issue + ds_read + split;
//  * the W DMA of tile kt + NSTAGE - 1 and the A loads of tile kt + 1 are issued between the
//    MFMAs of column blocks 0 and 1 (pinned by sched_barrier), not in a burst after the barrier.
// Synchronisation per K-tile kt (tile kt in stage kt % NSTAGE):
//   split A(kt) (hipcc waits for the A loads: vmcnt(0), nothing else is outstanding yet)
//   block 0: W DMA of tile kt + NSTAGE - 1 into stage (kt - 1) % NSTAGE (last read in tile
//            kt - 1, before the previous barrier); block 1: A loads of tile kt + 1
//   blocks ni: W fragments read two blocks ahead; with NSTAGE 3 blocks TN, TN + 1 are tile
//            kt + 1's first two, from its stage (landed and published by the previous barrier)
//   s_waitcnt vmcnt(2 TM) (this wave's W DMAs have landed, its A loads may still fly); s_barrier
// LDS image of W (per term, rows of 64 B, 16-B chunk q of row R stored at q ^ swzB(R)) as in
// conv_h3_kernel's 16x16x32 form: conflict-free ds_read_b128 for its lane groups.
#pragma once

#include "conv_h3_kernel.h"

namespace sfa {

typedef unsigned r3_u32x4 __attribute__((ext_vector_type(4)));

// Epilogues of the TRANSPOSED accumulator form (ABL 2048: the MFMAs take the W fragment as
// their A operand and the activation fragment as B, so the 16x16 tile of acc[mi][ni] holds
// C^T: lane l, register v -> output channel n0 + 16 ni + 4 (l >> 4) + v of pixel row
// m0 + 16 mi + (l & 15)). Every lane owns four consecutive channels of ONE pixel: its own row
// scale (no shuffle), float4 loads of bias / winv / residual and float4 stores of y (NHWC).
// RU: the residual may also be given at half resolution (a.res_up, the FPN skip convs), added
// bilinearly upsampled x2 (align_corners) exactly as res_up_sample evaluates it, 4 float4 taps
// per lane and column block (the 4 channels of the lane).
// The residual tile of r3t_epilogue_std in the transposed layout (lane: 4 channels of one row),
// loaded ahead of the epilogue by callers that can hide its latency behind their last MFMAs.
template <int TM, int TN>
__device__ __forceinline__ void r3t_res_load(const ConvArgs& a, x6_f32x4 (&rv)[TM][TN], int mrow0, int n0, int lane) {
  const int c16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int m = min(mrow0 + mi * 16 + c16, a.M - 1);
      rv[mi][ni] = *reinterpret_cast<const x6_f32x4*>(a.res + (size_t)m * a.N + n0 + ni * 16 + 4 * g);
    }
}

// PRE: the residual tile (a.res) was loaded by the caller (r3t_res_load) into `pre`, so its
// latency hid behind the MFMAs. CSL: the block's winv / bias columns n0 .. were staged in LDS by the
// caller (csb: [TN * 16] winv, then [TN * 16] bias, 0 without a bias) instead of read from global
// memory here (round 5: their latency was exposed at the end of every tile).
template <int TM, int TN, int NT, bool RU = false, bool PRE = false, bool CSL = false>
__device__ __forceinline__ void r3t_epilogue_std(const ConvArgs& a, f32x4_t (&acc)[TM][TN], unsigned char* smem,
                                                 int mrow0, int m0, int n0, int lane, const float (&ainv)[TM],
                                                 const x6_f32x4 (*pre)[TN] = nullptr, const float* csb = nullptr) {
  // every element is evaluated by the same rounding sequence (explicit fmaf, no contraction):
  // left to the compiler, the unrolled copies were contracted differently (some mul + add, some
  // fma, some packed), so a pixel's value depended on its row within the tile, i.e. on the
  // batch it was computed in
#pragma clang fp contract(off)
  const int M = a.M, c16 = lane & 15, g = lane >> 4;
  AmaxRows am(a.OH * a.OW, m0);
  x6_f32x4 rv[TM][TN];
  if (RU && a.res_up) {
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
      const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
      const float* r = a.res_up + (size_t)b * H * W * a.N;
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int n = n0 + ni * 16 + 4 * g;
        const x6_f32x4 a00 = *reinterpret_cast<const x6_f32x4*>(r + (size_t)(y0 * W + x0) * a.N + n);
        const x6_f32x4 a01 = *reinterpret_cast<const x6_f32x4*>(r + (size_t)(y0 * W + x1) * a.N + n);
        const x6_f32x4 a10 = *reinterpret_cast<const x6_f32x4*>(r + (size_t)(y1 * W + x0) * a.N + n);
        const x6_f32x4 a11 = *reinterpret_cast<const x6_f32x4*>(r + (size_t)(y1 * W + x1) * a.N + n);
#pragma unroll
        for (int v = 0; v < 4; ++v)
          rv[mi][ni][v] = fmaf(ly0, fmaf(lx0, a00[v], lx1 * a01[v]), ly1 * fmaf(lx0, a10[v], lx1 * a11[v]));
      }
    }
  }
  if (a.res) {
    if constexpr (PRE) {  // loaded by the caller (r3t_res_load)
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) rv[mi][ni] = pre[mi][ni];
    } else {
      r3t_res_load<TM, TN>(a, rv, mrow0, n0, lane);
    }
  }
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) {
    const int n = n0 + ni * 16 + 4 * g;
    x6_f32x4 cs, bn;
    if constexpr (CSL) {
      cs = *reinterpret_cast<const x6_f32x4*>(csb + ni * 16 + 4 * g);
      bn = *reinterpret_cast<const x6_f32x4*>(csb + TN * 16 + ni * 16 + 4 * g);
    } else {
      cs = *reinterpret_cast<const x6_f32x4*>(a.winv + n);
      bn = a.bias ? *reinterpret_cast<const x6_f32x4*>(a.bias + n) : x6_f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = mrow0 + mi * 16 + c16;
      x6_f32x4 val;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float t = fmaf(acc[mi][ni][v] * ainv[mi], cs[v], bn[v]);  // acc * ainv: exact (power of two)
        if (a.res || (RU && a.res_up)) t += rv[mi][ni][v];
        if (a.relu) t = fmaxf(t, 0.f);
        val[v] = t;
      }
      if (m < M) {
        *reinterpret_cast<x6_f32x4*>(a.y + (size_t)m * a.N + n) = val;
        if (a.amax_out)
          am.add(a.amax_out, m, fmaxf(fmaxf(fabsf(val[0]), fabsf(val[1])), fmaxf(fabsf(val[2]), fabsf(val[3]))));
      }
    }
  }
  if (a.amax_out) amax_commit_block<NT / 64>(a.amax_out, am.fb0, am.mx0, am.mx1, reinterpret_cast<float*>(smem));
}

// Heads (EPI_HEAD, transposed form): per head and pixel, ReLU(conv3x3 + b) of the lane's 16 of
// the head's 64 channels and the 1x1 conv's partial sums over them (4 outputs x TM pixels),
// reduced over the pixel's four lanes (l, l ^ 16, l ^ 32, l ^ 48) by v_permlane32/16_swap: each
// swap exchanges half of a pair of partials, so two levels leave lane l >> 4 = o with output o
// of each of its pixels (3 swaps + 3 adds per sub-tile, all VALU, no LDS, no barrier per head). The per-channel
// weight scale winv = 2^-e (fp16x3) is folded into the staged 1x1 weights and biases
// (w1 * winv, b / winv: exact power-of-two scalings), so T = max(acc * ainv + b', 0).
// The heads epilogue's constants for column tile nt (w1 * winv, bias / winv, the 1x1 biases) into LDS at
// HS: loads first, then the stores (the caller's barrier publishes them).  Round 5: staged once per
// block in the prologue, where the loads overlap the first W DMA, instead of after the K loop, where
// their L2 round trips (up to nine per tile before round 5) and a barrier sat between the last MFMAs
// and the first head products.
template <int NT, int HPB>
struct R3HeadStage {
  static constexpr int NI = (HPB * 256 + NT - 1) / NT, NJ = (HPB * 64 + NT - 1) / NT;
  static constexpr int BYTES = HPB * (256 + 64 + 4) * 4;
  float hv[NI], wv[NI], bv[NJ], bw[NJ], hb;
  __device__ __forceinline__ void load(const ConvArgs& a, int n0, int nt, int tid) {
    hb = a.hb1[nt * HPB * 4 + min(tid, HPB * 4 - 1)];
#pragma unroll
    for (int j = 0; j < NI; ++j) {  // indices clamped: no branch around the loads
      const int i = min(tid + j * NT, HPB * 256 - 1);
      hv[j] = a.hw1[nt * HPB * 256 + i];
      wv[j] = a.winv[n0 + (i >> 8) * 64 + (i & 63)];
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = min(tid + j * NT, HPB * 64 - 1);
      bv[j] = a.bias[n0 + i];
      bw[j] = a.winv[n0 + i];
    }
  }
  __device__ __forceinline__ void store(float* HS, int tid) const {
#pragma unroll
    for (int j = 0; j < NI; ++j)
      if (tid + j * NT < HPB * 256) HS[tid + j * NT] = hv[j] * wv[j];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      if (tid + j * NT < HPB * 64) HS[HPB * 256 + tid + j * NT] = bv[j] / bw[j];
    if (tid < HPB * 4) HS[HPB * 320 + tid] = hb;
  }
};

template <int TM, int TN, int NT, int HPB, bool PK = false>
__device__ __forceinline__ void r3t_epilogue_head(const ConvArgs& a, f32x4_t (&acc)[TM][TN], const unsigned char* smem,
                                                  int mrow0, int n0, int nt, int tid, const float (&ainv)[TM]) {
  const int M = a.M, lane = tid & 63, c16 = lane & 15, g = lane >> 4;
  // staged once per block in the prologue (r3_stage_head, its own LDS region: round 5)
  const float* WH = reinterpret_cast<const float*>(smem);  // [HPB][4][64]: w1 * winv
  const float* BP = WH + HPB * 256;                        // [HPB * 64]: bias / winv
  const float* HB = BP + HPB * 64;                         // [HPB][4]: the 1x1 convs' biases
  auto swap_add32 = [](float& x, float& y) {  // x: sum over (l, l^32) in lanes < 32; y: in lanes >= 32
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  };
  auto swap_add16 = [](float& x, float& y) {  // x: sum over (l, l^16) in even rows; y: odd rows
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  };
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
    float p[TM][4];
    if constexpr (PK) {
      // packed form: the activations t of a (column block, channel pair) as one float2, so the
      // bias fma and the 1x1 products run as v_pk_fma_f32 (2 lanes of work per VALU issue), and
      // only the head's ch outputs are formed (ch is wave-uniform: a scalar branch per output)
      using f2 = float __attribute__((ext_vector_type(2)));
      f2 T[TM][4][2];
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) {
        const int ni = 4 * hh + ci;
        const x6_f32x4 bp = *reinterpret_cast<const x6_f32x4*>(BP + hh * 64 + 16 * ci + 4 * g);
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f2 r = __builtin_elementwise_fma(f2{acc[mi][ni][2 * h], acc[mi][ni][2 * h + 1]},
                                                   f2{ainv[mi], ainv[mi]}, f2{bp[2 * h], bp[2 * h + 1]});
            T[mi][ci][h] = __builtin_elementwise_max(r, f2{0.f, 0.f});
          }
      }
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        if (o < ch) {
          f2 q[TM];
#pragma unroll
          for (int mi = 0; mi < TM; ++mi) q[mi] = f2{0.f, 0.f};
#pragma unroll
          for (int ci = 0; ci < 4; ++ci) {
            const x6_f32x4 w = *reinterpret_cast<const x6_f32x4*>(WH + hh * 256 + o * 64 + 16 * ci + 4 * g);
#pragma unroll
            for (int mi = 0; mi < TM; ++mi)
#pragma unroll
              for (int h = 0; h < 2; ++h)
                q[mi] = __builtin_elementwise_fma(T[mi][ci][h], f2{w[2 * h], w[2 * h + 1]}, q[mi]);
          }
#pragma unroll
          for (int mi = 0; mi < TM; ++mi) p[mi][o] = q[mi].x + q[mi].y;
        } else {
#pragma unroll
          for (int mi = 0; mi < TM; ++mi) p[mi][o] = 0.f;
        }
      }
    } else {
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int o = 0; o < 4; ++o) p[mi][o] = 0.f;
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) {
      const int ni = 4 * hh + ci;
      const int c = 16 * ci + 4 * g;  // channel within the head
      const x6_f32x4 bp = *reinterpret_cast<const x6_f32x4*>(BP + hh * 64 + c);
      x6_f32x4 w[4];
#pragma unroll
      for (int o = 0; o < 4; ++o) w[o] = *reinterpret_cast<const x6_f32x4*>(WH + hh * 256 + o * 64 + c);
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float t = fmaxf(fmaf(acc[mi][ni][v], ainv[mi], bp[v]), 0.f);
#pragma unroll
          for (int o = 0; o < 4; ++o) p[mi][o] = fmaf(t, w[o][v], p[mi][o]);
        }
    }
    }
    // level 1 (l ^ 32): lanes g < 2 keep outputs 0, 1, lanes g >= 2 outputs 2, 3
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      swap_add32(p[mi][0], p[mi][2]);
      swap_add32(p[mi][1], p[mi][3]);
    }
    // level 2 (l ^ 16): even rows keep the first of each pair, odd rows the second -> lane g: output g
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) swap_add16(p[mi][0], p[mi][1]);
    const float hb = HB[hh * 4 + g];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = mrow0 + mi * 16 + c16;
      if (g < ch && m < M) a.hout[(size_t)(hoff + g) * M + m] = p[mi][0] + hb;
    }
  }
}

// ABL: the product form's bits (round 4: the measured-and-rejected variants and ablations —
// compiler-scheduled DMA, A split one tile ahead, staggered split, 3-stage ring without the
// stagger, in-kernel split-K, non-temporal stores, residual prefetch, shifted A fragments, the
// grouped head launch — live in tools/experiments/r03/conv_r3_kernel.h with their convbench
// hooks). The values are kept from round 3, so the instances keep their names (conv.hip R3_*).
// Always set: 256 = spread the W DMA: A loads at block 0, then one W piece per block from block 2,
// the two waves of a SIMD (w, w + NW/2) on alternate blocks, so no SIMD issues two DMA bursts at
// once; 2048 = transposed accumulators (W fragment as the MFMA A operand) with the float4 /
// shuffle epilogues above.
// Per launch configuration:
// 4 = s_setprio 1 for the second half of the waves,
// 4096 = fp16 split in 2 VALU per value (split2h_x8, inline v_fma_mix),
// 8192 = W fragments read 3 column blocks ahead (with the stagger) instead of 2,
// 16384 = scalar tap decode + per-lane tap validity masks for the A addresses (one segment,
// C >= 32, checked at launch),
// 32768 = the epilogue also takes an upsampled half-resolution residual (a.res_up: the FPN skip
// convs; only those instances carry its registers),
// 65536 = (heads) packed epilogue: v_pk_fma_f32 over channel pairs, only the head's ch outputs
// formed,
// 524288 = channel-chunk-major K order over segment 0 (a 3x3 window, C % 32 == 0): K-tile kt covers
// tap kt % 9 of the 32-channel chunk kt / 9 (weight columns tap * C + 32 chunk .. +31), so the
// blocks resident on one XCD sweep a 32-channel slice of their input window through all 9 taps
// before the next slice: that slice (~1-2 MB per XCD for the heads) stays in the 4 MB L2, where
// the tap-major order's whole-window working set (4-9 MB per XCD at C = 128 / 256) re-read the
// input from the fabric at every tap (heads L0 / L1: 7x / 5x their input in HBM traffic),
// 2097152 = (with the stagger) the delayed half issues every W DMA piece of the K loop, the leading half none,
// 1048576 = half-tile stagger (NSTAGE 3): waves NW/2 .. NW - 1 run their K loop half a K-tile
// behind their SIMD partners (w - NW/2). The barrier that closes interval i (W of tile i + 1
// landed) comes after tile i for the first half of the waves and after the first half of tile i
// for the second, so the partners never reach their split VALU, their tile-top W reads and the
// barrier wait together: while one waits or splits, the other issues MFMAs. Interval i reads
// tiles i - 1 (second half only) and i, and DMAs tile i + 1: three stages. The delayed half reads
// the next tile's first W blocks ahead across its tile boundary (that tile was published by the
// barrier before); the leading half reads them after its barrier. Same products in the same
// order: bit-identical to the unstaggered loop.
// Without the stagger the ring has two stages (NSTAGE 2).
// The kernel body for output tile (and split-K slice) lbid; conv_r3_kernel maps blockIdx to lbid
// with xcd_remap.
template <int BM, int BN, int WM, int EPI, int OCC, int NSTAGE, int NSEG, int ABL = 0>
__device__ __forceinline__ void conv_r3_body(const ConvArgs& a, int lbid) {
  constexpr bool STAG = (ABL & 1048576) != 0;
  static_assert((ABL & (256 | 2048)) == (256 | 2048) &&
                    (ABL & ~(4 | 256 | 2048 | 4096 | 8192 | 16384 | 32768 | 65536 | 524288 | 1048576 | 2097152)) == 0,
                "product conv_r3 form (see the bit list)");
  static_assert(STAG ? NSTAGE == 3 : NSTAGE == 2, "W ring depth: 3 stages with the stagger, else 2");
  static_assert(NSEG == 1 || NSEG == 2, "segments");
  static_assert(EPI == EPI_STD || EPI == EPI_HEAD, "epilogue");
  constexpr int NW = BM / WM, NT = NW * 64;
  constexpr int TM = WM / 16, TN = BN / 16;
  constexpr int BK = 32, BROW = BK * 2;  // W row bytes per term
  constexpr int TERM_B = BN * BROW, STAGE = 2 * TERM_B;
  constexpr int ND_BT = TERM_B / 1024, ND_B = 2 * ND_BT;  // 1-KiB DMA pieces (16 rows each)
  constexpr int NB = (ND_B + NW - 1) / NW;
  constexpr int NB_REM = ND_B % NW;  // if != 0: waves < NB_REM issue NB pieces, the rest NB - 1
  static_assert(BM % WM == 0 && WM % 16 == 0 && BN % 16 == 0 && TERM_B % 1024 == 0, "tile");
  static_assert(TN >= 2, "two W blocks in flight");
  // heads: the epilogue's constants in their own region after the W stages (R3HeadStage)
  constexpr int HS_OFF = NSTAGE * STAGE;
  // standard epilogue: the tile's winv / bias columns in LDS after the W stages (round 5: read per column
  // block from global memory they sat behind the previous block's stores)
  constexpr int EPI_BYTES = EPI == EPI_HEAD ? HS_OFF + R3HeadStage<NT, BN / 64>::BYTES : HS_OFF + 2 * BN * 4;
  constexpr int LDS_BYTES = NSTAGE * STAGE > EPI_BYTES ? NSTAGE * STAGE : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];

  auto swzB = [](int R) { return ((R >> 2) & 3) ^ ((((R & 15) + 4) >> 3) & 1); };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, g = lane >> 4;
  const int n_tiles = a.N / BN;
  const int m_tiles = (a.M + BM - 1) / BM;
  const int nsplit = a.ksplit > 1 ? a.ksplit : 1;
  const int kz = lbid / (m_tiles * n_tiles);  // split-K slice of this block
  lbid -= kz * (m_tiles * n_tiles);
  const int mt = lbid / n_tiles, nt = lbid - mt * n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int M = a.M;
  // heads: the epilogue's constants in flight during the whole prologue (stored before its barrier)
  [[maybe_unused]] R3HeadStage<NT, BN / 64> hst;
  if constexpr (EPI == EPI_HEAD) hst.load(a, n0, nt, tid);
  constexpr int NCS = EPI == EPI_HEAD ? 1 : (2 * BN + NT - 1) / NT;  // winv / bias entries per thread
  [[maybe_unused]] float csb_v[NCS];
  if constexpr (EPI != EPI_HEAD) {
#pragma unroll
    for (int j = 0; j < NCS; ++j) {
      const int i = tid + j * NT;
      csb_v[j] = i < BN ? a.winv[n0 + i] : (i < 2 * BN && a.bias ? a.bias[n0 + i - BN] : 0.f);
    }
  }

  // ---- A: this lane's rows (one per 16-row sub-tile), gather origins per segment ----
  // (round 5: row decomposition by multiply-high divisions, a.fd_ow / a.fd_oh from the launch)
  int r_pix[NSEG][TM], r_ihw[NSEG][TM];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    const int m = m0 + wave * WM + mi * 16 + c16;
    const bool ok = m < M;
    const int mm = ok ? m : 0;
    const int t = fast_div(mm, a.fd_ow), ow = mm - t * a.OW;
    const int b = fast_div(t, a.fd_oh), oh = t - b * a.OH;
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
      const ConvSeg& sgm = a.seg[sg];
      const int ih = ok ? oh * sgm.stride - sgm.pad : -16384;
      const int iw = ow * sgm.stride - sgm.pad;
      r_pix[sg][mi] = (b * sgm.H + ih) * sgm.W + iw;
      r_ihw[sg][mi] = (ih << 16) | (iw & 0xffff);
    }
  }
  const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.seg[0].x), (short)0, (int)a.seg[0].bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.seg[NSEG - 1].x), (short)0, (int)a.seg[NSEG - 1].bytes, 0x00020000);

  // ---- W DMA slots: pieces e = wave + NW * j (term e / ND_BT, rows (e % ND_BT) * 16 + lane / 4) ----
  const int wst = a.wstride ? a.wstride : a.Kpad;  // row stride of the fp16 terms
  const unsigned term_bytes = (unsigned)a.N * (unsigned)wst * 2u;
  const __amdgpu_buffer_rsrc_t rsw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.wh), (short)0, (int)(2 * term_bytes), 0x00020000);
  // row R = 16 (e % ND_BT) + lane / 4 of piece e has swzB(R) = swzB(lane / 4), so the lane part
  // of the source offset is the same for every piece and the piece part is wave-uniform
  // (one VGPR for all NB pieces; a non-constant soffset operand of the LDS-DMA builtin makes
  // hipcc's host pass drop the kernel stub, so the uniform part is added to the VGPR offset)
  const int wlane = (((n0 + lane / 4) * wst + a.wk0 + 8 * ((lane % 4) ^ swzB(lane / 4))) << 1);
  int boff_s[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int e = wave + NW * j < ND_B ? wave + NW * j : ND_B - 1;
    boff_s[j] = (int)((e / ND_BT) * term_bytes) + (e % ND_BT) * 16 * wst * 2;  // uniform: wave, j, args
  }

  // fp16x3 scale of the frame of this lane's A row in each 16-row sub-tile: the block's first two
  // frames' scales by uniform loads, rows of later frames (small maps) their own
  float as[TM];  // 1 / as (exact: powers of two) is recomputed for the epilogue
  {
    const int P = a.OH * a.OW, f0 = m0 / P, fb = (f0 + 1) * P;
    float sinv, sA, sB;
    amax_frame_scale2(a.amax_in, NSEG, f0, min(f0 + 1, (M - 1) / P), sA, sinv, sB, sinv);
    if (fb >= M) sB = sA;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = min(m0 + wave * WM + mi * 16 + c16, M - 1);
      if (m < fb) as[mi] = sA;
      else if (m < fb + P) as[mi] = sB;
      else as[mi] = amax_frame_scale(a.amax_in, NSEG, m / P, sinv);
    }
  }

  r3_u32x4 raw[TM][2];  // A fragment of the next K-tile (f32 bits)
  // ABL 16384 (one segment, C >= 32: a K-tile lies in one tap): the tap decode is wave-uniform
  // (scalar), and each lane keeps a validity bit per tap and sub-tile row and the byte offset of
  // its pixel + channel group, so an A address costs a bit test, an add and a select.
  constexpr bool FAST_A = (ABL & 16384) != 0 && NSEG == 1;  // two-segment launches are refused
  // chunk-major K order over segment 0 (a 3x3 window, checked at launch); segment 1 (the fused
  // 1x1 downsample) keeps its order after it
  constexpr bool CMAJ = (ABL & 524288) != 0;
  const int cmaj_tiles = NSEG == 2 ? a.kseg1 / BK : a.Kpad / BK;  // K-tiles of segment 0
  // first weight column of K-tile kt: tap * C + chunk * 32 (chunk-major) or kt * BK
  auto kcol = [&](int kt) -> int {
    if constexpr (CMAJ) {
      if (NSEG == 1 || kt < cmaj_tiles) {
        const int chunk = (kt * 7282) >> 16;  // kt / 9 for kt < 3640 (checked at launch)
        return (kt - 9 * chunk) * a.seg[0].C + chunk * BK;
      }
    }
    return kt * BK;
  };

  unsigned vmask[TM], abase[TM];
  if constexpr (FAST_A) {
    const ConvSeg& sg0 = a.seg[0];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int ih = r_ihw[0][mi] >> 16;
      const int iw = (int)(short)(r_ihw[0][mi] & 0xffff);
      unsigned msk = 0;
      for (int t = 0; t < sg0.taps && t < 32; ++t) {
        const int kh = (t * sg0.kdiv_mul) >> sg0.kdiv_sh, kw = t - kh * sg0.KW;
        if ((unsigned)(ih + kh) < (unsigned)sg0.H && (unsigned)(iw + kw) < (unsigned)sg0.W) msk |= 1u << t;
      }
      vmask[mi] = msk;
      abase[mi] = (unsigned)(((r_pix[0][mi] << sg0.logC) + 8 * g) << 2);
    }
  }
  auto load_a_fast = [&](int k0) {
    const ConvSeg& sg0 = a.seg[0];
    const int tap = k0 >> sg0.logC, c0 = k0 & (sg0.C - 1);
    const int kh = (tap * sg0.kdiv_mul) >> sg0.kdiv_sh, kw = tap - kh * sg0.KW;
    const unsigned toff = (unsigned)((((kh * sg0.W + kw) << sg0.logC) + c0) << 2);
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const bool ok = tap < 32 && ((vmask[mi] >> tap) & 1u);
      const unsigned off = ok ? abase[mi] + toff : 0x80000000u;
      raw[mi][0] = __builtin_amdgcn_raw_buffer_load_b128(rs0, off, 0, 0);
      raw[mi][1] = __builtin_amdgcn_raw_buffer_load_b128(rs0, off + 16u, 0, 0);
    }
  };
  auto load_a_seg = [&](auto sgc, const __amdgpu_buffer_rsrc_t rs, int kl) {
    constexpr int SG = decltype(sgc)::value;
    const ConvSeg& sgm = a.seg[SG];
    const int kk = kl + 8 * g;
    const int tap = kk >> sgm.logC;
    const int c = kk & (sgm.C - 1);
    const int kh = (tap * sgm.kdiv_mul) >> sgm.kdiv_sh;
    const int kw = tap - kh * sgm.KW;
    const bool tap_ok = tap < sgm.taps;
    const int toff = kh * sgm.W + kw;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int ih = r_ihw[SG][mi] >> 16;
      const int iw = (int)(short)(r_ihw[SG][mi] & 0xffff);
      const bool ok = tap_ok & ((unsigned)(ih + kh) < (unsigned)sgm.H) & ((unsigned)(iw + kw) < (unsigned)sgm.W);
      const unsigned off = ok ? (unsigned)((((r_pix[SG][mi] + toff) << sgm.logC) + c) << 2) : 0x80000000u;
      raw[mi][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
      raw[mi][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16u, 0, 0);
    }
  };
  auto load_a = [&](int kt) {
    const int k0 = kcol(kt);
    if constexpr (FAST_A) {
      load_a_fast(k0);
    } else if constexpr (NSEG == 2) {
      if (k0 >= a.kseg1)
        load_a_seg(std::integral_constant<int, 1>(), rs1, k0 - a.kseg1);
      else
        load_a_seg(std::integral_constant<int, 0>(), rs0, k0);
    } else {
      load_a_seg(std::integral_constant<int, 0>(), rs0, k0);
    }
  };
  auto load_w_piece = [&](int j, int kt, unsigned char* S) {
    if (NB_REM == 0 || j < NB - 1 || wave < NB_REM)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsw, (__attribute__((address_space(3))) void*)(S + (wave + NW * j) * 1024), 16,
          (unsigned)(wlane + boff_s[j] + 2 * kcol(kt)), 0, 0, 0);
  };
  auto load_w = [&](int kt, unsigned char* S) {
#pragma unroll
    for (int j = 0; j < NB; ++j) load_w_piece(j, kt, S);
  };
  // ABL 2097152 (with the stagger; round 5): the delayed half also issues its SIMD partner's W pieces in
  // the K loop (piece e = wave - NW / 2 + NW j), the leading half none: the delayed half (s_setprio 1)
  // reached each barrier ~1,100 cycles early and idled there, the leading half now sheds its DMA issue
  // (heads -2.2 %, same bits: profiles/r05ah_*)
  constexpr bool DMA_DEL = (ABL & 2097152) != 0;
  [[maybe_unused]] int boff_p[NB];
  if constexpr (DMA_DEL) {
    static_assert(NB_REM == 0, "whole pieces per wave");
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int e = (wave >= NW / 2 ? wave - NW / 2 : wave) + NW * j;
      boff_p[j] = (int)((e / ND_BT) * term_bytes) + (e % ND_BT) * 16 * wst * 2;
    }
  }
  auto load_w_piece_p = [&](int j, int kt, unsigned char* S) {
    const int e = wave - NW / 2 + NW * j;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(S + e * 1024), 16,
                                             (unsigned)(wlane + boff_p[j] + 2 * kcol(kt)), 0, 0, 0);
  };
  f16x8_t hf[2][TM];  // split A of this K-tile
  auto split_a = [&](f16x8_t (&h)[2][TM]) {
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      if constexpr ((ABL & 4096) != 0) {  // 2 VALU per value (split2h_x8)
        split2h_x8(__builtin_bit_cast(x6_f32x4, raw[mi][0]), __builtin_bit_cast(x6_f32x4, raw[mi][1]), as[mi],
                   h[0][mi], h[1][mi]);
      } else {
        f16x4_t t0, t1, u0, u1;
        split2h(__builtin_bit_cast(x6_f32x4, raw[mi][0]), as[mi], t0, t1);
        split2h(__builtin_bit_cast(x6_f32x4, raw[mi][1]), as[mi], u0, u1);
        h[0][mi] = __builtin_shufflevector(t0, u0, 0, 1, 2, 3, 4, 5, 6, 7);
        h[1][mi] = __builtin_shufflevector(t1, u1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[mi][ni][v] = 0.f;

  const int bfo = c16 * BROW + ((g ^ swzB(c16)) << 4);  // this lane's W fragment in a block
  constexpr int RA = (ABL & 8192) != 0 ? 3 : 2;  // W fragment blocks read ahead of their MFMAs
  constexpr int RS = RA + 1;
  static_assert(RA == 2 || STAG, "3-block read-ahead: with the stagger only");
  static_assert(!STAG || (TN % RS == 0 && TN % 2 == 0 && TN / 2 > RA), "stagger: W ring slots must repeat per tile");
  f16x8_t bq[RS][2];  // W fragment ring: block p in slot p % RS
  auto read_b = [&](const unsigned char* S, int ni, f16x8_t (&dst)[2]) {
    dst[0] = *reinterpret_cast<const f16x8_t*>(S + bfo + ni * 16 * BROW);
    dst[1] = *reinterpret_cast<const f16x8_t*>(S + TERM_B + bfo + ni * 16 * BROW);
  };

  const int nk = a.Kpad / BK / nsplit;  // this block's K-tiles: kt0 .. kt0 + nk - 1
  const int kt0 = kz * nk;
  constexpr int NA_OPS = 2 * TM;  // A loads per K-tile (issued after the tile's W DMA)
  // prologue: W tile 0 (the stagger's first interval DMAs tile 1), A tile 0; this wave's W
  // landed, then everyone's
  // (heads: the epilogue's constants, loaded at the top of the body, stored here once they land and
  // published by this barrier)
  if (nk > 0) load_w(kt0, smem);
  load_a(kt0);
  if constexpr (EPI == EPI_HEAD) hst.store(reinterpret_cast<float*>(smem + HS_OFF), tid);
  else {
#pragma unroll
    for (int j = 0; j < NCS; ++j)
      if (tid + j * NT < 2 * BN) reinterpret_cast<float*>(smem + HS_OFF)[tid + j * NT] = csb_v[j];
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NA_OPS) : "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr ((ABL & 4) != 0) {
    if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }
  const int wave_half = wave >= NW / 2 ? 1 : 0;  // SIMD partners: waves w and w + NW / 2
  auto mma_block = [&](int ni) {
    const f16x8_t c0 = bq[ni % RS][0], c1 = bq[ni % RS][1];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      f32x4_t cc = acc[mi][ni];
      cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[1][mi], cc, 0, 0, 0);
      cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c1, hf[0][mi], cc, 0, 0, 0);
      cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[0][mi], cc, 0, 0, 0);
      acc[mi][ni] = cc;
    }
  };
  // stagger (see the ABL list): the K loop of one half of the waves, HB = the delayed half.
  // Interval i = the steps between barriers i - 1 and i; a block's interval-relative position r
  // places the W DMA pieces (slot s at r = 2 + 2 s + HB, as ABL 256 spreads them) of tile i + 1.
  auto stag_loop = [&](auto hb_c) {
    constexpr bool HB = decltype(hb_c)::value;
    constexpr int H2 = TN / 2;
    constexpr int SLOTS = (TN - 2) / 2 >= 1 ? (TN - 2) / 2 : 1;
    constexpr int PPB = (NB + SLOTS - 1) / SLOTS;
    auto dma_slot = [&](int s, int tile, unsigned char* S) {
#pragma unroll
      for (int jj = 0; jj < PPB; ++jj) {
        const int j = s * PPB + jj;
        if (j < NB) {
          if constexpr (DMA_DEL) {
            if constexpr (HB) {
              load_w_piece(j, tile, S);
              load_w_piece_p(j, tile, S);
            }
          } else {
            load_w_piece(j, tile, S);
          }
        }
      }
    };
    int st_cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const unsigned char* S = smem + st_cur * STAGE;
      const int st_n1 = st_cur + 1 == NSTAGE ? 0 : st_cur + 1;
      const int st_n2 = st_n1 + 1 == NSTAGE ? 0 : st_n1 + 1;
      const bool more_a = kt + 1 < nk;
      split_a(hf);
      __builtin_amdgcn_sched_barrier(0);
      if (!HB || kt == 0) {
#pragma unroll
        for (int p = 0; p < RA; ++p) read_b(S, p, bq[p % RS]);
      }
      if (HB && kt == 0 && more_a) {
        // the delayed half's pieces of tile 1 whose slots fall before its first tile (r < H2)
#pragma unroll
        for (int s = 0; s < SLOTS; ++s)
          if (3 + 2 * s < H2) dma_slot(s, kt0 + 1, smem + st_n1 * STAGE);
      }
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        if (ni == 0 && more_a) load_a(kt0 + kt + 1);
        {
          const bool late = HB && ni >= H2;                   // block in interval kt + 1
          const int r = HB ? (late ? ni - H2 : ni + H2) : ni;  // compile-time for each HB
          const int tw = late ? kt + 2 : kt + 1;               // tile DMA'd in this interval
          if (r >= 2 && ((r - 2) & 1) == (HB ? 1 : 0) && ((r - 2) >> 1) < SLOTS && tw < nk)
            dma_slot((r - 2) >> 1, kt0 + tw, smem + (late ? st_n2 : st_n1) * STAGE);
        }
        const int p = ni + RA;
        if (p < TN)
          read_b(S, p, bq[p % RS]);
        else if (HB && more_a)
          read_b(smem + st_n1 * STAGE, p - TN, bq[p % RS]);
        mma_block(ni);
        if (ni == (HB ? H2 - 1 : TN - 1)) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      st_cur = st_n1;
    }
  };
  if constexpr (STAG) {
    if (wave_half)
      stag_loop(std::true_type{});
    else
      stag_loop(std::false_type{});
  }
  // unstaggered loop (NSTAGE 2): PPB W pieces per issuing block; blocks 2, 4, .. for one half of
  // the waves, 3, 5, .. for the other
  constexpr int SLOTS2 = (TN - 2) / 2 >= 1 ? (TN - 2) / 2 : 1;
  constexpr int PPB2 = (NB + SLOTS2 - 1) / SLOTS2;
  static_assert(TN >= 4, "spread DMA needs 4 column blocks");
  int st_cur = 0;
  for (int kt = 0; kt < (STAG ? 0 : nk); ++kt) {
    const unsigned char* S = smem + st_cur * STAGE;
    const int st_nx = st_cur ^ 1;  // the stage of tile kt + 1 (last read in tile kt - 1)
    const bool more = kt + 1 < nk;
    split_a(hf);
    // keep the W DMA below the split: hipcc's wait for the A loads would otherwise also wait
    // for DMAs issued just before it (it counts the conditional DMA path conservatively)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int p = 0; p < RA; ++p) read_b(S, p, bq[p]);
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      if (ni == 0 && more) load_a(kt0 + kt + 1);
      if (ni >= 2 && ((ni - 2) >> 1) * PPB2 < NB && more && wave_half == (ni & 1)) {
#pragma unroll
        for (int jj = 0; jj < PPB2; ++jj) {
          const int j = ((ni - 2) >> 1) * PPB2 + jj;
          if (j < NB) load_w_piece(j, kt0 + kt + 1, smem + st_nx * STAGE);
        }
      }
      const int p = ni + RA;
      if (p < TN) read_b(S, p, bq[p % RS]);
      mma_block(ni);
      __builtin_amdgcn_sched_barrier(0);
    }
    // this wave's W DMAs of tile kt + 1 and A loads have landed, then everyone's: that stage is
    // readable, and this tile's stage is free for the next DMA
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    st_cur = st_nx;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float ainv[TM];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) ainv[mi] = 1.f / as[mi];
  if (nsplit > 1) {  // split-K partials, transposed form: float4 per lane (the reduce launch adds them)
    float* part = a.part + (size_t)kz * M * a.N;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int m = m0 + wave * WM + mi * 16 + c16, n = n0 + ni * 16 + 4 * g;
        const x6_f32x4 cs = *reinterpret_cast<const x6_f32x4*>(a.winv + n);
        x6_f32x4 val;
#pragma unroll
        for (int v = 0; v < 4; ++v) val[v] = acc[mi][ni][v] * ainv[mi] * cs[v];
        if (m < M) *reinterpret_cast<x6_f32x4*>(part + (size_t)m * a.N + n) = val;
      }
    return;
  }
  if constexpr (EPI == EPI_HEAD) {  // reads only the constants' region: no barrier after the K loop
    r3t_epilogue_head<TM, TN, NT, BN / 64, (ABL & 65536) != 0>(a, acc, smem + HS_OFF, m0 + wave * WM, n0, nt, tid,
                                                              ainv);
  } else {
    __syncthreads();
    r3t_epilogue_std<TM, TN, NT, (ABL & 32768) != 0, false, true>(a, acc, smem, m0 + wave * WM, m0, n0, lane, ainv,
                                                                  nullptr, reinterpret_cast<const float*>(smem + HS_OFF));
  }
}

template <int BM, int BN, int WM, int EPI, int OCC, int NSTAGE, int NSEG, int ABL = 0>
__global__ void __launch_bounds__((BM / WM) * 64, OCC) conv_r3_kernel(const ConvArgs a) {
  conv_r3_body<BM, BN, WM, EPI, OCC, NSTAGE, NSEG, ABL>(a, xcd_remap(blockIdx.x, gridDim.x));
}

// Launch-time checks of one conv_r3 launch (the kernel never bounds-checks these).
template <int BM, int BN, int EPI, int ABL>
inline int conv_r3_check(const ConvArgs& a) {
  if (!a.wh || !a.winv || a.Kpad % 32 != 0 || (a.nseg == 2 && a.kseg1 % 32 != 0) || a.N % BN != 0 ||
      (a.res_up && ((ABL & 32768) == 0 || a.res || a.nseg != 1))) {
    set_error("conv_r3: K/N not aligned to the tile, no split weights or an upsampled residual (Kpad=%d kseg1=%d N=%d)", a.Kpad,
              a.kseg1, a.N);
    return SFA_E_UNSUPPORTED;
  }
  if ((ABL & 16384) != 0 && (a.nseg != 1 || a.seg[0].C < 32 || a.seg[0].taps > 32)) {
    set_error("conv_r3: fast A addressing needs one segment with C >= 32 (C=%d)", a.seg[0].C);
    return SFA_E_UNSUPPORTED;
  }
  if ((ABL & 524288) != 0 && (a.seg[0].taps != 9 || a.seg[0].C % 32 != 0 ||
                              (a.nseg == 2 ? a.kseg1 : a.Kpad) != 9 * a.seg[0].C || a.Kpad / 32 > 3600 ||
                              a.wstride || a.wk0)) {
    set_error("conv_r3: chunk-major K order needs a 3x3 first segment with C %% 32 == 0 (C=%d Kpad=%d)", a.seg[0].C,
              a.Kpad);
    return SFA_E_UNSUPPORTED;
  }
  for (int s = 0; s < a.nseg; ++s)
    if (a.seg[s].C < 8) {  // a lane's 8 k values must be 8 channels of one input pixel
      set_error("conv_r3: segment %d has C=%d < 8", s, a.seg[s].C);
      return SFA_E_UNSUPPORTED;
    }
  if (a.wstride && (a.wstride < a.wk0 + a.Kpad || a.wk0 % 8 != 0)) {
    set_error("conv_r3: K slice [%d, %d) outside the weight rows (stride %d)", a.wk0, a.wk0 + a.Kpad, a.wstride);
    return SFA_E_INVALID;
  }
  if (2ull * a.N * (a.wstride ? a.wstride : a.Kpad) * 2ull >= (1ull << 31)) {
    set_error("conv_r3: split weights >= 2 GiB");
    return SFA_E_UNSUPPORTED;
  }
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  if (ks > 1 && (EPI != EPI_STD || (a.Kpad / 32) % ks != 0 || !a.part ||
                 (size_t)ks * a.M * a.N > a.part_floats || a.N % 4 != 0)) {
    set_error("conv_r3: split-K %d unsupported here (Kpad=%d N=%d)", ks, a.Kpad, a.N);
    return SFA_E_UNSUPPORTED;
  }
  return SFA_OK;
}

template <int BM, int BN, int WM, int EPI, int OCC, int NSTAGE, int ABL = 0>
inline int launch_conv_r3_cfg(const ConvArgs& a, hipStream_t st) {
  const int crc = conv_r3_check<BM, BN, EPI, ABL>(a);
  if (crc != SFA_OK) return crc;
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  const long long nblocks = (long long)ceil_div(a.M, BM) * (a.N / BN) * ks;
  if (nblocks <= 0 || nblocks > 0x7fffffffll) {
    set_error("conv_r3: bad grid (M=%d N=%d)", a.M, a.N);
    return SFA_E_INVALID;
  }
  ConvArgs b = a;  // the row decomposition's multiply-high divisions
  b.fd_ow = make_fast_div((unsigned)a.OW);
  b.fd_oh = make_fast_div((unsigned)a.OH);
  if (a.nseg == 2)
    hipLaunchKernelGGL((conv_r3_kernel<BM, BN, WM, EPI, OCC, NSTAGE, 2, ABL>), dim3((unsigned)nblocks),
                       dim3((BM / WM) * 64), 0, st, b);
  else
    hipLaunchKernelGGL((conv_r3_kernel<BM, BN, WM, EPI, OCC, NSTAGE, 1, ABL>), dim3((unsigned)nblocks),
                       dim3((BM / WM) * 64), 0, st, b);
  SFA_LAUNCH_CHECK();
  if (ks > 1) {  // the slices' partials combined by the reduce launch
    const long long nel = (long long)a.M * a.N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((nel + 1023) / 1024)), dim3(256), 0, st, a);
    SFA_LAUNCH_CHECK();
  }
  return SFA_OK;
}

}  // namespace sfa
