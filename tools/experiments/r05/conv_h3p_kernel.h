// 3x3 / stride-1 / pad-1 body convolutions (fpn_resnet.py:42-71 BasicBlock conv1 / conv2 of layer1-4),
// fp16x3, PERSISTENT form of the strip kernel (round 5; measured and NOT adopted: bit-identical, but
// layer1 +5 %, layer2 +22 %, layers 3 / 4 -1..2 % per launch and the bench -3 %,
// profiles/r05b_convbench5_persistent_strip.txt — the per-tile prologue / epilogue is not what limits the
// strip kernel; tools/convbench5.hip keeps the hook).
//
// Same products, K order, operand split, LDS images and epilogue arithmetic as conv_h3s_kernel with
// the pre-split strip (ABL 4): bit-identical outputs.  What differs is the life of a workgroup.  The
// strip kernel runs one 128-row output tile per workgroup, so every tile pays a prologue (row
// decomposition with integer divisions, per-lane frame-scale loads, the first strip + W DMA and its
// full latency before the first MFMA) and an epilogue drain (residual, stores, the per-frame maxima)
// during which the workgroup's slot does no MFMA work; with K = 576 (layer1) a tile has only 18
// k-steps to amortise them (ablation: no epilogue -17 %, profiles/r03p_convbench_strip_ablations.txt).
// Here grid = CUs x blocks per CU and each workgroup walks its units (output tile x split-K slice)
// u = lb, lb + G, ... (lb = the XCD-aware logical block: an XCD's workgroups hold a contiguous range of
// units each round, so the 3x3 halo rows stay in its L2).  The k-step pipeline runs straight across
// unit boundaries: the next unit's first strip is DMA'd during this unit's last super-step (kw 1, with
// this unit's residual tile) and its first W tile at the last k-step, so the epilogue overlaps them;
// the unit geometry is uniform scalar work and the per-lane row math uses multiply-high divisions by
// host-computed magic numbers (FastDiv) instead of the compiler's generic 32-bit division sequences.
// Units may span at most two frames (frame >= BM rows): the frame scales are two per unit, read with
// uniform loads.  The epilogue's amax reduction uses two LDS buffers alternating by unit.
#pragma once

#include "../../../lidar-image_object-detection_-fpn_resnet-yolov8_amd/csrc/conv_h3s_kernel.h"

namespace sfa {

// FastDiv / make_fast_div / fast_div: conv.h (the product's copy since round 5)
inline FastDiv make_fastdiv(unsigned d) { return make_fast_div(d); }
__device__ __forceinline__ int fdiv(int n, FastDiv f) { return fast_div(n, f); }

struct H3pArgs {
  int units;      // m_tiles * n_tiles * nsplit
  int mn_tiles;   // m_tiles * n_tiles
  int n_tiles;
  int nsl;        // super-steps (kh, 32-channel chunk) per unit: 3 * C / 32 / nsplit
  int lognchunk;  // log2(C / 32)
  FastDiv fW, fH, fP, fMN, fNT;
};

template <int BM, int BN, int WM, int OCC, bool RESPF>
__global__ void __launch_bounds__((BM / WM) * 64, OCC) conv_h3p_kernel(const ConvArgs a, const H3pArgs q) {
  constexpr int NW = BM / WM;
  constexpr int TM = WM / 16, TN = BN / 16;
  constexpr int AROW = 128, BROW = 64;  // bytes per LDS row: 32 f32 / 32 fp16
  constexpr int SROWS = BM + 2;          // strip rows m0 - 1 .. m0 + BM
  constexpr int ND_S = (SROWS + 7) / 8;  // strip DMA pieces (8 rows each)
  constexpr int S_BYTES = ND_S * 1024;
  constexpr int TERM_B = BN * BROW, W_BYTES = 2 * TERM_B;
  constexpr int ND_B = W_BYTES / 1024;  // W pieces per k-step (16 rows each)
  constexpr int NS = (ND_S + NW - 1) / NW, NS_REM = ND_S % NW;
  constexpr int NB = (ND_B + NW - 1) / NW, NB_REM = ND_B % NW;
  constexpr int PROWS = WM + 2;               // a wave's pre-split rows (its WM rows + the kw halo)
  constexpr int PR_BYTES = (PROWS + 1) * 64;  // per term: 32 fp16 per row, + one zero row
  constexpr int W_OFF = S_BYTES, P_OFF = S_BYTES + 2 * W_BYTES, RED_OFF = P_OFF + NW * 2 * PR_BYTES;
  constexpr int LDS_BYTES = RED_OFF + 2 * 2 * NW * 4;
  static_assert(NW % 2 == 0 && WM % 16 == 0 && BN % 16 == 0, "tile");
  static_assert(OCC * LDS_BYTES <= 160 * 1024, "blocks per CU vs LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];

  auto swzA = [](int R) { return ((R >> 1) & 7) ^ ((((R & 15) + 4) >> 2) & 2); };
  auto swzB = [](int R) { return ((R >> 2) & 3) ^ ((((R & 15) + 4) >> 3) & 1); };
  auto swzP = [](int R) { return ((R >> 2) & 1) << 1; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  const int lb = xcd_remap(blockIdx.x, G);
  if (lb >= q.units) return;  // uniform
  const int M = a.M, N = a.N;
  const ConvSeg& g = a.seg[0];
  const int H = g.H, W = g.W, P = a.OH * a.OW;
  const int nchunk = 1 << q.lognchunk;
  const bool wave_full_ns = NS_REM == 0 || wave < NS_REM;  // this wave's strip pieces: NS or NS - 1

  // fixed per-lane strip piece rows j = 8 (wave + NW i) + lane / 8 and the W piece offsets
  const int srow = lane >> 3;
  const int kq = (lane & 7) ^ swzA(8 * wave + srow);
  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.x), (short)0, (int)g.bytes, 0x00020000);
  const unsigned term_bytes = (unsigned)N * (unsigned)a.Kpad * 2u;
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.wh), (short)0,
                                                                       (int)(2 * term_bytes), 0x00020000);
  // W piece e = wave + NW jj holds rows 16 (e % (ND_B / 2)) + lane / 4 of term e / (ND_B / 2); the
  // pieces of one wave differ by whole 16-row groups (the swizzle repeats every 16 rows), so one
  // per-lane offset + a uniform delta per piece
  static_assert(NW % 4 == 0 || NB == 1, "W piece deltas");
  const int bof0 = [&] {
    const int R = wave * 16 + (lane >> 2);
    return (int)((R * a.Kpad + 8 * ((lane & 3) ^ swzB(R))) << 1);
  }();
  auto bdelta = [&](int jj) {  // uniform
    const int e = wave + NW * jj < ND_B ? wave + NW * jj : ND_B - 1;
    const int term = e / (ND_B / 2);
    return (int)(term * term_bytes) + (((e - term * (ND_B / 2)) - wave) * 16 * a.Kpad << 1);
  };
  const int c16 = lane & 15, gq = lane >> 4;
  unsigned char* const WB = smem + W_OFF;
  unsigned char* const PH = smem + P_OFF + wave * 2 * PR_BYTES;  // hi rows, lo + PR_BYTES
  float* const RED = reinterpret_cast<float*>(smem + RED_OFF);
  if (lane < 8)  // the zero rows (conv padding at kw 0 / 2)
    *reinterpret_cast<x6_f32x4*>(PH + (lane & 4 ? PR_BYTES : 0) + PROWS * 64 + (lane & 3) * 16) =
        x6_f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- unit context (uniform) + per-lane rows
  struct Unit {
    int kz, m0, n0, s0, fb;
    float sA, sB;
  };
  auto unit_of = [&](int u) {
    Unit c;
    c.kz = fdiv(u, q.fMN);
    const int rest = u - c.kz * q.mn_tiles;
    const int mt = fdiv(rest, q.fNT);
    c.m0 = mt * BM;
    c.n0 = (rest - mt * q.n_tiles) * BN;
    c.s0 = c.kz * q.nsl;
    const int f0 = fdiv(c.m0, q.fP);
    c.fb = (f0 + 1) * P;  // first row of the next frame
    float t;
    c.sA = amax_frame_scale(a.amax_in, 1, f0, t);
    c.sB = c.fb < M ? amax_frame_scale(a.amax_in, 1, f0 + 1, t) : c.sA;
    return c;
  };
  // strip row validity: bit 3 i + kh = strip piece i's row (image row y) has input row y + kh - 1
  // inside the image (rows outside the map: no bit)
  static_assert(3 * NS <= 32, "validity bits");
  auto strip_rows = [&](int m0) {
    unsigned bits = 0;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int j = 8 * (wave + NW * i) + srow;
      const int m = m0 - 1 + j;
      const bool ok = j < SROWS && m >= 0 && m < M;
      const int t = fdiv(ok ? m : 0, q.fW);
      const int y = t - fdiv(t, q.fH) * H;
      const unsigned v = (y > 0 ? 1u : 0u) | 2u | (y < H - 1 ? 4u : 0u);
      bits |= ok ? v << (3 * i) : 0u;
    }
    return bits;
  };
  auto load_strip = [&](int m0, unsigned sy, int s) {
    const int kh = s >> q.lognchunk, c0 = (s & (nchunk - 1)) << 5;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      if (NS_REM == 0 || i < NS - 1 || wave < NS_REM) {
        const int m = m0 - 1 + 8 * (wave + NW * i) + srow;
        const bool ok = (sy >> (3 * i + kh)) & 1u;
        const unsigned off = ok ? (unsigned)((((m + (kh - 1) * W) << g.logC) + c0 + 4 * kq) << 2) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsx, (__attribute__((address_space(3))) void*)(smem + (wave + NW * i) * 1024), 16, off, 0, 0, 0);
      }
    }
  };
  auto wk0 = [&](int s, int kw) {  // K offset of the W tile of super-step s, tap kw
    const int kh = s >> q.lognchunk, c0 = (s & (nchunk - 1)) << 5;
    return (kh * 3 + kw) * g.C + c0;
  };
  auto load_w = [&](int n0, int k0, unsigned char* S) {
    const int base = (int)((n0 * a.Kpad + k0) << 1);
#pragma unroll
    for (int jj = 0; jj < NB; ++jj) {
      if (NB_REM == 0 || jj < NB - 1 || wave < NB_REM)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsw, (__attribute__((address_space(3))) void*)(S + (wave + NW * jj) * 1024), 16,
            (unsigned)(bof0 + base + bdelta(jj)), 0, 0, 0);
    }
  };
  // waits for this wave's vector-memory operations but the `younger` most recent ones (immediates)
  auto wait_vm = [&](int younger_ns, bool plus_res) {
    // younger_ns: strip pieces issued after the awaited W tile (0 or this wave's count)
    if (!younger_ns) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (!plus_res) {
      if (wave_full_ns) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS - 1) : "memory");
    } else {
      if (wave_full_ns) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS + TM * TN) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NS - 1 + TM * TN) : "memory");
    }
  };

  Unit cu = unit_of(lb);
  unsigned sy = strip_rows(cu.m0);
  const int nsplit = q.units / q.mn_tiles;

  f32x4_t acc[TM][TN];
  x6_f32x4 rvp[TM][TN];  // RESPF: the residual tile, loaded during the last super-step

  auto presplit = [&](const Unit& c) {
    const int rr = lane >> 3, qq = lane & 7;
    constexpr int NP = (PROWS + 7) / 8, NP0 = (NP + 1) / 2;  // reads in two groups (VGPR budget)
    auto rd = [&](int p) {
      const int r = 8 * p + rr;
      const int j = wave * WM + (r < PROWS ? r : 0);
      return *reinterpret_cast<const x6_f32x4*>(smem + j * AROW + ((qq ^ swzA(j)) << 4));
    };
    auto wr = [&](int p, const x6_f32x4 x) {
      const int r = 8 * p + rr;
      if (r < PROWS) {
        const int j = wave * WM + r;
        const float sc = c.m0 - 1 + j >= c.fb ? c.sB : c.sA;
        const int off = r * 64 + (((qq >> 1) ^ swzP(r)) << 4) + (qq & 1) * 8;
        typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
        unsigned h0, h1, l0, l1;
        split2h_pair(x[0], x[1], sc, h0, l0);
        split2h_pair(x[2], x[3], sc, h1, l1);
        *reinterpret_cast<u32x2_t*>(PH + off) = u32x2_t{h0, h1};
        *reinterpret_cast<u32x2_t*>(PH + PR_BYTES + off) = u32x2_t{l0, l1};
      }
    };
    x6_f32x4 x[NP0];
#pragma unroll
    for (int p = 0; p < NP0; ++p) x[p] = rd(p);
#pragma unroll
    for (int p = 0; p < NP0; ++p) wr(p, x[p]);
#pragma unroll
    for (int p = NP0; p < NP; ++p) x[p - NP0] = rd(p);
#pragma unroll
    for (int p = NP0; p < NP; ++p) wr(p, x[p - NP0]);
  };
  int xm[TM];
  auto lane_rows = [&](const Unit& c) {
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = min(c.m0 + wave * WM + mi * 16 + c16, M - 1);
      xm[mi] = m - fdiv(m, q.fW) * W;
    }
  };
  // the epilogue's row scales 1 / s of the unit's (at most two) frames
  auto row_ainv = [&](const Unit& c, float (&ainv)[TM]) {
    float tA, tB;
    (void)amax_frame_scale(a.amax_in, 1, fdiv(c.m0, q.fP), tA);
    tB = tA;
    if (c.fb < M) (void)amax_frame_scale(a.amax_in, 1, fdiv(c.m0, q.fP) + 1, tB);
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) ainv[mi] = min(c.m0 + wave * WM + mi * 16 + c16, M - 1) >= c.fb ? tB : tA;
  };
  auto compute = [&](const unsigned char* Sw, int kw) {
    f16x8_t hf[2][TM];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const bool pad = kw == 0 ? xm[mi] == 0 : (kw == 2 ? xm[mi] == W - 1 : false);
      const int R = pad ? PROWS : mi * 16 + c16 + kw;
      const int o = R * 64 + ((gq ^ swzP(R)) << 4);
      hf[0][mi] = *reinterpret_cast<const f16x8_t*>(PH + o);
      hf[1][mi] = *reinterpret_cast<const f16x8_t*>(PH + PR_BYTES + o);
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

  // prologue: the first unit's strip and W tile
  load_strip(cu.m0, sy, cu.s0);
  load_w(cu.n0, wk0(cu.s0, 0), WB);
  int t = 0;  // k-steps issued so far (W stage parity), continuous across units
  const bool res_pf = RESPF && a.res && nsplit == 1;
  for (int k = 0;; ++k) {
    const int un = lb + (k + 1) * G;
    const bool has_next = un < q.units;
    Unit nu = cu;
    unsigned nsy = sy;
    lane_rows(cu);
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int sl = 0; sl < q.nsl; ++sl) {
      const int s = cu.s0 + sl;
      const bool last = sl + 1 == q.nsl;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        // kw 2: W(t) landed (the strip issued after it at kw 1, and in the last super-step the
        // residual loads before that strip, may still fly); kw 0 / 1: everything landed
        if (kw == 2) wait_vm(1, last && res_pf);
        else wait_vm(0, false);
        __builtin_amdgcn_s_barrier();
        unsigned char* const wdst = WB + ((t + 1) & 1) * W_BYTES;
        if (kw < 2) load_w(cu.n0, wk0(s, kw + 1), wdst);
        else if (!last) load_w(cu.n0, wk0(s + 1, 0), wdst);
        else if (has_next) load_w(nu.n0, wk0(nu.s0, 0), wdst);
        else load_w(cu.n0, wk0(s, 2), wdst);  // no next unit: a harmless reload keeps the counts uniform
        if (kw == 1) {
          if (!last) {
            load_strip(cu.m0, sy, s + 1);  // every wave has split strip s (barrier above)
          } else {
            if (res_pf) {  // buffer loads: 32-bit offsets, rows past M read 0 (never stored)
              const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
                  const_cast<float*>(a.res), (short)0, (int)((size_t)M * N * 4 < 0x7fffffffu ? (size_t)M * N * 4 : 0x7fffffffu),
                  0x00020000);
#pragma unroll
              for (int mi = 0; mi < TM; ++mi) {
                const int m = cu.m0 + wave * WM + mi * 16 + c16;
                const unsigned o = m < M ? (unsigned)((m * N + cu.n0 + 4 * gq) * 4) : 0x80000000u;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni)
                  rvp[mi][ni] = __builtin_bit_cast(x6_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                 rsr, o == 0x80000000u ? o : o + ni * 64u, 0, 0));
              }
            }
            if (has_next) {
              nu = unit_of(un);
              nsy = strip_rows(nu.m0);
              load_strip(nu.m0, nsy, nu.s0);
            } else {
              load_strip(cu.m0, sy, s);
            }
          }
        }
        if (kw == 0) presplit(cu);
        compute(WB + (t & 1) * W_BYTES, kw);
        ++t;
      }
    }
    asm volatile("" ::: "memory");
    float ainv[TM];
    row_ainv(cu, ainv);
    if (nsplit > 1) {  // split-K partials, transposed form: float4 per lane (the reduce launch adds them)
      float* part = a.part + (size_t)cu.kz * M * N;
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int m = cu.m0 + wave * WM + mi * 16 + c16, n = cu.n0 + ni * 16 + 4 * gq;
          const x6_f32x4 cs = *reinterpret_cast<const x6_f32x4*>(a.winv + n);
          x6_f32x4 val;
#pragma unroll
          for (int v = 0; v < 4; ++v) val[v] = acc[mi][ni][v] * ainv[mi] * cs[v];
          if (m < M) *reinterpret_cast<x6_f32x4*>(part + (size_t)m * N + n) = val;
        }
    } else {
      r3t_epilogue_std<TM, TN, NW * 64, false, RESPF>(a, acc, reinterpret_cast<unsigned char*>(RED + (k & 1) * 2 * NW),
                                                     cu.m0 + wave * WM, cu.m0, cu.n0, lane, ainv, rvp);
    }
    if (!has_next) break;
    cu = nu;
    sy = nsy;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup exits
}

// Host side: the persistent strip conv when its preconditions hold (one-segment 3x3/s1/p1, C a
// multiple of 32, frames of >= BM rows), SFA_E_UNSUPPORTED otherwise.
template <int BM, int BN, int WM, int OCC, bool RESPF>
inline int launch_conv_h3p_cfg(const ConvArgs& a, hipStream_t st) {
  const ConvSeg& g = a.seg[0];
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  if (!a.wh || !a.winv || a.nseg != 1 || g.KH != 3 || g.KW != 3 || g.stride != 1 || g.pad != 1 || g.C < 32 ||
      (g.C & 31) != 0 || a.Kpad != 9 * g.C || a.OH != g.H || a.OW != g.W || a.N % BN != 0 ||
      a.OH * a.OW < BM || a.M % (a.OH * a.OW) != 0 || a.wstride || a.wk0 || a.res_up) {
    set_error("conv_h3p: not a one-segment 3x3/s1/p1 conv with C %% 32 == 0 and frames >= %d rows", BM);
    return SFA_E_UNSUPPORTED;
  }
  if (ks > 1 && ((3 * (g.C >> 5)) % ks != 0 || !a.part || (size_t)ks * a.M * a.N > a.part_floats || a.N % 4 != 0)) {
    set_error("conv_h3p: split-K %d unsupported here (C=%d N=%d)", ks, g.C, a.N);
    return SFA_E_UNSUPPORTED;
  }
  if (2ull * a.N * a.Kpad * 2ull >= (1ull << 31)) {
    set_error("conv_h3p: split weights >= 2 GiB");
    return SFA_E_UNSUPPORTED;
  }
  const int m_tiles = ceil_div(a.M, BM), n_tiles = a.N / BN;
  const long long units = (long long)m_tiles * n_tiles * ks;
  if (units <= 0 || units > 0x7fffffffll) {
    set_error("conv_h3p: bad grid (M=%d N=%d)", a.M, a.N);
    return SFA_E_INVALID;
  }
  H3pArgs q;
  q.units = (int)units;
  q.mn_tiles = m_tiles * n_tiles;
  q.n_tiles = n_tiles;
  q.nsl = 3 * (g.C >> 5) / ks;
  q.lognchunk = ilog2(g.C >> 5);
  q.fW = make_fastdiv((unsigned)g.W);
  q.fH = make_fastdiv((unsigned)g.H);
  q.fP = make_fastdiv((unsigned)(a.OH * a.OW));
  q.fMN = make_fastdiv((unsigned)q.mn_tiles);
  q.fNT = make_fastdiv((unsigned)n_tiles);
  const int slots = cu_count(st) * OCC;
  const int grid = q.units < slots ? q.units : slots;
  hipLaunchKernelGGL((conv_h3p_kernel<BM, BN, WM, OCC, RESPF>), dim3((unsigned)grid), dim3((BM / WM) * 64), 0, st, a,
                     q);
  SFA_LAUNCH_CHECK();
  if (ks > 1) {  // the slices' partials combined by the reduce launch
    const long long nel = (long long)a.M * a.N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((nel + 1023) / 1024)), dim3(256), 0, st, a);
    SFA_LAUNCH_CHECK();
  }
  return SFA_OK;
}

}  // namespace sfa
