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

// Product form (round 4: the measured-and-rejected variants and ablations live in
// tools/experiments/r03/conv_h3s_kernel.h with their convbench hooks): transposed accumulators
// (the W fragment as the MFMA A operand) with conv_r3_kernel.h's float4 epilogue
// (r3t_epilogue_std) and float4 split-K partials, the fp16 split in 2 VALU per value
// (split2h_x8 / split2h_pair, inline v_fma_mix). ABL bits (the values are kept from round 3, so
// the instances keep their names: H3S_64 = 142, H3S_128 = 10 in conv.hip):
// 4 = pre-split strip: at kw 0 each wave splits ITS rows of the f32 strip (WM + 2 rows, the kw
// halo included) once into fp16 hi / lo rows of a private LDS region, and the three kw k-steps
// read ready fp16 fragments (a third of the split VALU; conv padding by reading a zero row).
// One f32 strip buffer: the next strip is issued at kw 1, when every wave has split this one.
// 128 = (with 4) the residual tile loaded at the last super-step's kw 1 (in place of the no-op
// strip reload), so the last six k-steps' MFMAs hide its latency; 2 and 8 are always set.
// 256 = register-staged W (round 4): each k-step's W pieces are fetched with buffer_load_dwordx4
// into VGPRs at the step's start and written to the other W stage with ds_write_b128 after the
// step's MFMAs (an LDS-DMA piece costs ~60 issue cycles, a load + ds_write_b128 ~20); same
// LDS image, same products: bit-identical.
// 1024 = (with 4; round 5) the strip into REGISTERS: each wave loads its own WM + 2 rows (the kw halo) of
// the next (kh, chunk) strip with buffer loads at kw 1 and splits them from its VGPRs at kw 0, so the f32
// strip never passes through LDS (no strip buffer, no LDS-DMA pieces, no f32 LDS reads in the split).
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
  constexpr bool PS = (ABL & 4) != 0;
  constexpr bool RESPF = PS && (ABL & 128) != 0;
  constexpr bool RW = (ABL & 256) != 0;
  constexpr bool SREG = (ABL & 1024) != 0;
  constexpr int PROWS = WM + 2;              // a wave's pre-split rows (its WM rows + the kw halo)
  constexpr int PR_BYTES = (PROWS + 1) * 64;  // per term: 32 fp16 per row, + one zero row
  constexpr int NSB = PS ? (SREG ? 0 : 1) : 2;  // f32 strip buffers
  constexpr int NP = (PROWS + 7) / 8;         // PS: pre-split row groups per wave (8 rows x 8 lanes)
  constexpr int MAIN_BYTES = NSB * S_BYTES + 2 * W_BYTES + (PS ? NW * 2 * PR_BYTES : 0);
  constexpr int CSB_OFF = MAIN_BYTES;  // the tile's winv / bias columns (epilogue), staged in the prologue
  constexpr int LDS_BYTES = MAIN_BYTES + 2 * BN * 4;
  static_assert(NW % 2 == 0 && WM % 16 == 0 && BN % 16 == 0, "tile");
  static_assert((ABL & 10) == 10 && (ABL & ~(2 | 4 | 8 | 128 | 256 | 1024)) == 0, "product strip-kernel form (see the bit list)");
  static_assert(!SREG || (PS && !RW), "strip in registers: the pre-split form, W by LDS-DMA");
  static_assert(EPI == EPI_STD, "transposed form: standard epilogue only");
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

  // strip pieces d = wave + NW * i: rows 8d + lane / 8 (d of the wave's parity: one swizzle). Row j
  // is input pixel m = m0 - 1 + j itself (stride 1, same geometry): its byte offset at channel 4 kq,
  // and in bit 3 i + kh whether input row y(m) + kh - 1 lies in the image (no bit: outside the map).
  // Round 5: y(m) by multiply-high divisions (a.fd_w / a.fd_h, host magic numbers), the super-step's
  // (kh, chunk) offset one uniform add per piece (profiles/r05g_*: the strip prologue and the per-piece
  // address arithmetic were 13 % and ~25 % of a layer1 wave's time).
  const int srow = lane >> 3;
  const int kq = (lane & 7) ^ swzA(8 * wave + srow);
  static_assert(3 * NS <= 32 && 3 * NP <= 32, "3 row-validity bits per strip piece / pre-split group in one word");
  int s_base[NS];
  unsigned s_ok = 0;
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const int j = 8 * (wave + NW * i) + srow;
    const int m = m0 - 1 + j;
    const bool ok = j < SROWS && m >= 0 && m < M;
    const int t = fast_div(ok ? m : 0, a.fd_w);
    const int y = t - fast_div(t, a.fd_h) * H;
    s_base[i] = ((m << g.logC) + 4 * kq) << 2;
    s_ok |= ok ? ((y > 0 ? 1u : 0u) | 2u | (y < H - 1 ? 4u : 0u)) << (3 * i) : 0u;
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
  auto swzP = [](int R) { return ((R >> 2) & 1) << 1; };  // conflict-free at every kw row offset

  // SREG: this lane's pre-split rows r = 8 p + lane / 8 of the wave (strip row wave WM + r, input pixel
  // m0 - 1 + wave WM + r), channels 4 (lane & 7) .. + 3 of the chunk: byte offset and kh validity bits
  [[maybe_unused]] int p_base[NP];
  [[maybe_unused]] unsigned p_ok = 0;
  if constexpr (SREG) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int r = 8 * p + (lane >> 3);
      const int m = m0 - 1 + wave * WM + r;
      const bool ok = r < PROWS && m >= 0 && m < M;
      const int t = fast_div(ok ? m : 0, a.fd_w);
      const int y = t - fast_div(t, a.fd_h) * H;
      p_base[p] = ((m << g.logC) + 4 * (lane & 7)) << 2;
      p_ok |= ok ? ((y > 0 ? 1u : 0u) | 2u | (y < H - 1 ? 4u : 0u)) << (3 * p) : 0u;
    }
  }
  const int lognchunk = g.logC - 5, nchunk = 1 << lognchunk;
  const int nsl = 3 * nchunk / nsplit;  // this block's (kh, chunk) super-steps s0 .. s0 + nsl - 1
  const int s0 = kz * nsl;
  auto load_strip = [&](int s, unsigned char* S) {
    const int kh = s >> lognchunk, c0 = (s & (nchunk - 1)) << 5;
    const int delta = ((((kh - 1) * W) << g.logC) + c0) << 2;  // uniform
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      if (NS_REM == 0 || i < NS - 1 || wave < NS_REM) {
        const bool ok = (s_ok >> (3 * i + kh)) & 1u;
        const unsigned off = ok ? (unsigned)(s_base[i] + delta) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsx, (__attribute__((address_space(3))) void*)(S + (wave + NW * i) * 1024), 16, off, 0, 0, 0);
      }
    }
  };
  [[maybe_unused]] x6_f32x4 xs[NP];  // SREG: the next strip's rows
  auto load_strip_regs = [&](int s) {
    const int kh = s >> lognchunk, c0 = (s & (nchunk - 1)) << 5;
    const int delta = ((((kh - 1) * W) << g.logC) + c0) << 2;  // uniform
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const bool ok = (p_ok >> (3 * p + kh)) & 1u;
      const unsigned off = ok ? (unsigned)(p_base[p] + delta) : 0x80000000u;
      xs[p] = __builtin_bit_cast(x6_f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0));
    }
  };
  auto load_w = [&](int k0, unsigned char* S) {
#pragma unroll
    for (int jj = 0; jj < NB; ++jj) {
      if (NB_REM == 0 || jj < NB - 1 || wave < NB_REM)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsw, (__attribute__((address_space(3))) void*)(S + (wave + NW * jj) * 1024), 16,
            (unsigned)(boff[jj] + 2 * k0), 0, 0, 0);
    }
  };
  // the fp16x3 scales of the block's first two frames (uniform loads); x of this lane's A row in each
  // 16-row tile (kw edge masks) and its frame's scale — rows of later frames (blocks taller than a
  // frame: small maps) read their own
  const int P = a.OH * a.OW;
  const int f0 = m0 / P;
  const int fb = (f0 + 1) * P;  // first row of the next frame
  // both frames' words loaded at once (the second frame clamped into the batch; used only if it exists)
  float sA, iA, sB, iB;
  amax_frame_scale2(a.amax_in, 1, f0, min(f0 + 1, (M - 1) / P), sA, iA, sB, iB);
  if (fb >= M) {
    sB = sA;
    iB = iA;
  }
  const int c16 = lane & 15, gq = lane >> 4;
  int xm[TM];
  float as[TM], ainv[TM];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    const int m = min(m0 + wave * WM + mi * 16 + c16, M - 1);
    xm[mi] = m - fast_div(m, a.fd_w) * W;
    if (m < fb) {
      as[mi] = sA;
      ainv[mi] = iA;
    } else if (m < fb + P) {
      as[mi] = sB;
      ainv[mi] = iB;
    } else {
      as[mi] = amax_frame_scale(a.amax_in, 1, m / P, ainv[mi]);
    }
  }
  x6_u32x4 wreg[NB];  // RW: the next k-step's W pieces
  auto load_w_regs = [&](int k0) {
#pragma unroll
    for (int jj = 0; jj < NB; ++jj) {
      if (NB_REM == 0 || jj < NB - 1 || wave < NB_REM)
        wreg[jj] = __builtin_amdgcn_raw_buffer_load_b128(rsw, (unsigned)(boff[jj] + 2 * k0), 0, 0);
    }
  };
  auto store_w_regs = [&](unsigned char* S) {
#pragma unroll
    for (int jj = 0; jj < NB; ++jj) {
      if (NB_REM == 0 || jj < NB - 1 || wave < NB_REM)
        *reinterpret_cast<x6_u32x4*>(S + (wave + NW * jj) * 1024 + lane * 16) = wreg[jj];
    }
  };
  // RW: wait for this wave's W loads (every vector-memory op issued after them may still fly)
  auto wait_w_regs = [&](int younger) {
    if (younger == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (NS_REM == 0 || wave < NS_REM) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS - 1) : "memory");
  };
  auto wk0 = [&](int s, int kw) {  // K offset of the W tile of super-step s, tap kw
    const int kh = s >> lognchunk, c0 = (s & (nchunk - 1)) << 5;
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
    // every row's read first: one LDS latency, not one per row (the compiler cannot tell the strip
    // reads from the pre-split writes apart and waits after each read otherwise; profiles/r05g_*)
    x6_f32x4 xr[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int r = 8 * p + rr, j = wave * WM + (r < PROWS ? r : 0);
      if constexpr (SREG) xr[p] = xs[p];
      else xr[p] = *reinterpret_cast<const x6_f32x4*>(Ss + j * AROW + ((q ^ swzA(j)) << 4));
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int r = 8 * p + rr;
      if (r < PROWS) {
        const int j = wave * WM + r;
        const x6_f32x4 x = xr[p];
        const float sc = m0 - 1 + j >= fb ? sB : sA;
        const int off = r * 64 + (((q >> 1) ^ swzP(r)) << 4) + (q & 1) * 8;
        typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
        unsigned h0, h1, l0, l1;
        split2h_pair(x[0], x[1], sc, h0, l0);
        split2h_pair(x[2], x[3], sc, h1, l1);
        *reinterpret_cast<u32x2_t*>(PH + off) = u32x2_t{h0, h1};
        *reinterpret_cast<u32x2_t*>(PH + PR_BYTES + off) = u32x2_t{l0, l1};
      }
    }
  };
  // the epilogue's winv / bias columns: loaded here, written to LDS after the first k-step (their
  // latency hidden by it), read after the K loop's later barriers
  float* const CSB = reinterpret_cast<float*>(smem + CSB_OFF);
  static_assert(2 * BN <= NT, "one winv / bias value per thread");
  const float csb_v = tid < BN ? a.winv[n0 + tid] : (tid < 2 * BN && a.bias ? a.bias[n0 + tid - BN] : 0.f);
  if constexpr (PS) {  // the zero rows (conv padding at kw 0 / 2)
    if (lane < 8) *reinterpret_cast<x6_f32x4*>(PH + (lane & 4 ? PR_BYTES : 0) + PROWS * 64 + (lane & 3) * 16) =
        x6_f32x4{0.f, 0.f, 0.f, 0.f};
  }
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
      split2h_x8(q0, q1, as[mi], hf[0][mi], hf[1][mi]);
    }
  };
  auto compute = [&](const unsigned char* Ss, const unsigned char* Sw, int kw) {
    f16x8_t hf[2][TM];
    read_a(Ss, kw, hf);
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
      if (ni + 2 < TN) read_b(ni + 2);
      const f16x8_t c0 = bq[ni % 3][0], c1 = bq[ni % 3][1];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        f32x4_t cc = acc[mi][ni];
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[1][mi], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c1, hf[0][mi], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[0][mi], cc, 0, 0, 0);
        acc[mi][ni] = cc;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  unsigned char* const WB = smem + NSB * S_BYTES;
  if constexpr (RW) {
    load_w_regs(wk0(s0, 0));
    load_strip(s0, smem);
    wait_w_regs(1);
    store_w_regs(WB);
  } else if constexpr (SREG) {
    load_strip_regs(s0);
    load_w(wk0(s0, 0), WB);
  } else {
    load_strip(s0, smem);
    load_w(wk0(s0, 0), WB);
  }
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
          } else if (SREG)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NP) : "memory");
          else if (NS_REM == 0 || wave < NS_REM)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS - 1) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if constexpr (RW) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // W(t) stores
        __builtin_amdgcn_s_barrier();
        const int wnext = kw < 2 ? wk0(s, kw + 1) : (last ? wk0(s, 2) : wk0(s + 1, 0));
        unsigned char* const wdst = WB + ((t + 1) & 1) * W_BYTES;
        if constexpr (RW) load_w_regs(wnext);
        else load_w(wnext, wdst);
        bool strip_after = false;
        if (kw == 1) {
          if (RESPF && last) {  // the residual tile (the last MFMAs hide its latency)
            if (a.res && nsplit == 1) r3t_res_load<TM, TN>(a, rvp, m0 + wave * WM, n0, lane);
          } else {
            if constexpr (SREG) load_strip_regs(last ? s : s + 1);  // this wave has split strip s
            else load_strip(last ? s : s + 1, smem);                 // every wave has split strip s
            strip_after = true;
          }
        }
        if (kw == 0) presplit(smem);
        compute(smem, WB + (t & 1) * W_BYTES, kw);
        if (t == 0 && tid < 2 * BN) CSB[tid] = csb_v;
        if constexpr (RW) {
          if (RESPF && last && kw == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          else wait_w_regs(strip_after ? 1 : 0);
          store_w_regs(wdst);
        }
        continue;
      }
      if (kw == 1) {
        if (NS_REM == 0 || wave < NS_REM)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS - 1) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if constexpr (RW) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // W(t) stores
      __builtin_amdgcn_s_barrier();  // W(t) (and the strip) landed for every wave; W(t-1) no longer read
      const int wnext = kw < 2 ? wk0(s, kw + 1) : (last ? wk0(s, 2) : wk0(s + 1, 0));
      unsigned char* const wdst = WB + ((t + 1) & 1) * W_BYTES;
      unsigned char* const sdst = smem + ((sl + 1) & 1) * S_BYTES;
      if constexpr (RW) load_w_regs(wnext);
      else load_w(wnext, wdst);
      if (kw == 0) load_strip(last ? s : s + 1, sdst);
      compute(smem + (sl & 1) * S_BYTES, WB + (t & 1) * W_BYTES, kw);
      if (t == 0 && tid < 2 * BN) CSB[tid] = csb_v;
      if constexpr (RW) {
        wait_w_regs(kw == 0 ? 1 : 0);
        store_w_regs(wdst);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (nsplit > 1) {  // split-K partials, transposed form: float4 per lane
    // combined by the reduce launch, or (ConvArgs::tile_cnt) by the last slice to finish
    // (splitk_ticket, conv_h3_kernel.h: sc1 partial stores, one ticket per tile)
    const __amdgpu_buffer_rsrc_t rsp = __builtin_amdgcn_make_buffer_rsrc(
        a.part, (short)0, (int)((size_t)nsplit * M * a.N * 4 < 0x7fffffffu ? (size_t)nsplit * M * a.N * 4 : 0x7fffffffu),
        0x00020000);
    const bool tk = a.tile_cnt != nullptr;
    x6_f32x4 val[TM][TN];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int m = m0 + wave * WM + mi * 16 + c16, n = n0 + ni * 16 + 4 * gq;
        // winv from the LDS copy (a global load here sat behind the previous partial's store)
        const x6_f32x4 cs = *reinterpret_cast<const x6_f32x4*>(CSB + ni * 16 + 4 * gq);
#pragma unroll
        for (int v = 0; v < 4; ++v) val[mi][ni][v] = acc[mi][ni][v] * ainv[mi] * cs[v];
        if (m < M) {
          const unsigned off = (unsigned)((((size_t)kz * M + m) * a.N + n) * 4);
          if (tk) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(x6_u32x4, val[mi][ni]), rsp, off, 0, 16);
          else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(x6_u32x4, val[mi][ni]), rsp, off, 0, 0);
        }
      }
    if (!tk || !splitk_ticket(a.tile_cnt, mt * n_tiles + nt, nsplit, reinterpret_cast<unsigned*>(smem + 1024)))
      return;
    // the last slice: splitk_reduce_kernel's epilogue on this tile (slice order, + bias, + residual, ReLU)
    AmaxRows am(a.OH * a.OW, m0);
    // per 16-row sub-tile: the row's slice partials and residual loaded for every column block
    // first, then summed in slice order and stored (round 5: loaded per block they sat behind the
    // previous block's store, one round trip each); bias from the LDS copy
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = m0 + wave * WM + mi * 16 + c16;
      const bool mok = m < M;
      const int mm = mok ? m : M - 1;
      x6_f32x4 sv[TN], rr[TN];
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int n = n0 + ni * 16 + 4 * gq;
        auto part_z = [&](int z) {
          return z == kz ? val[mi][ni]
                         : __builtin_bit_cast(x6_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                            rsp, (unsigned)((((size_t)z * M + mm) * a.N + n) * 4), 0, 16));
        };
        sv[ni] = part_z(0);
        for (int z = 1; z < nsplit; ++z) sv[ni] += part_z(z);
        rr[ni] = a.res ? *reinterpret_cast<const x6_f32x4*>(a.res + (size_t)mm * a.N + n) : x6_f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int n = n0 + ni * 16 + 4 * gq;
        x6_f32x4 t = sv[ni] + *reinterpret_cast<const x6_f32x4*>(CSB + BN + ni * 16 + 4 * gq);
        if (a.res) t += rr[ni];
        if (a.relu) {
#pragma unroll
          for (int v = 0; v < 4; ++v) t[v] = fmaxf(t[v], 0.f);
        }
        if (mok) {
          *reinterpret_cast<x6_f32x4*>(a.y + (size_t)m * a.N + n) = t;
          if (a.amax_out) am.add(a.amax_out, m, fmaxf(fmaxf(fabsf(t[0]), fabsf(t[1])), fmaxf(fabsf(t[2]), fabsf(t[3]))));
        }
      }
    }
    if (a.amax_out) amax_commit_block<NT / 64>(a.amax_out, am.fb0, am.mx0, am.mx1, reinterpret_cast<float*>(smem));
    return;
  }
  __syncthreads();
  r3t_epilogue_std<TM, TN, NT, false, RESPF, true>(a, acc, smem, m0 + wave * WM, m0, n0, lane, ainv, rvp, CSB);
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
  ConvArgs b = a;  // the strip rows' multiply-high divisions
  b.fd_w = make_fast_div((unsigned)g.W);
  b.fd_h = make_fast_div((unsigned)g.H);
  // tickets only with one word per output tile in the array: else the reduce launch
  if (ks == 1 || (long long)ceil_div(a.M, BM) * (a.N / BN) > (long long)a.tile_cnt_words) b.tile_cnt = nullptr;
  hipLaunchKernelGGL((conv_h3s_kernel<BM, BN, WM, EPI, OCC, ABL>), dim3((unsigned)nblocks), dim3((BM / WM) * 64), 0,
                     st, b);
  SFA_LAUNCH_CHECK();
  if (ks > 1 && !b.tile_cnt) {  // the slices' partials combined by the reduce launch
    const long long nel = (long long)a.M * a.N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((nel + 1023) / 1024)), dim3(256), 0, st, a);
    SFA_LAUNCH_CHECK();
  }
  return SFA_OK;
}

}  // namespace sfa
