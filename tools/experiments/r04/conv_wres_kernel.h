// 3x3 / stride-1 / pad-1 convolution with the WHOLE weight matrix resident in LDS, fp16x3 on
// v_mfma_f32_16x16x32_f16 (gfx950 / CDNA4): the 64-wide layer1 convs (C = N = 64, K = 576).
//
// The strip kernel (conv_h3s_kernel.h) streams every weight K-tile from L2 into an LDS ring once
// per 128-row tile (147 KB per tile: 8 LDS-DMA pieces per k-step) and synchronises its waves
// with a barrier per k-step. Here a persistent block (one per CU) DMAs the split weights once
// (18 K-tiles x 2 fp16 terms x 64 rows x 64 B = 147,456 B, conv_r3_kernel's swizzled stage
// image per K-tile), and from then on every wave works alone: it walks its own 32-row output
// units, loads each K-tile's A fragment straight into VGPRs (conv_r3_kernel's register-A form:
// one input pixel, 8 channels, 32 B per lane and 16-row sub-tile) PD K-tiles ahead, splits it
// into fp16 hi / lo and multiplies against W fragments read from the resident image. No W
// traffic, no DMA and no barrier after the prologue; the last K-tiles of a unit already load
// the first A fragments of the wave's next unit, and the residual tile is loaded ahead of the
// epilogue. The frame maxima of the output are committed per wave (no block reduction).
// Bits: the same products, per-element K order and epilogue rounding as the strip kernel
// (K-tile t = super-step (kh, 32-channel chunk) t / 3, tap kw = t % 3; hi*lo, lo*hi, hi*hi per
// K-tile; r3t_epilogue_std's fmaf sequence), so its output equals conv_h3s_kernel's bit for bit.
//
// Round 4, measured and NOT adopted (tools/convbench4, profiles/r04t_convbench4_layer1_wres.txt):
// bit-identical to the strip kernel, but 156.6-157.2 us against its 118.7-120.4 us (8 waves, A
// prefetch 1 or 2 K-tiles ahead; 12 waves spill). With N = 64 a K-tile's A fragment feeds only 24
// MFMAs per wave, and the register-A form loads it once per tap (4 buffer_load_dwordx4 per wave and
// K-tile, three times the strip kernel's A traffic): the vector-memory path, not the W staging it
// removes, sets the pace.
#pragma once

#include "conv_r3_kernel.h"  // (-I<pkg>/csrc)

namespace sfa {

namespace wres {
constexpr int BN = 64, BK = 32, BROW = 64;       // W: 64 columns, 32 K per tile, 64-B rows
constexpr int TERM_B = BN * BROW, STAGE = 2 * TERM_B;  // one K-tile, two fp16 terms: 8 KiB
constexpr int WM = 32, TM = WM / 16, TN = BN / 16;     // a wave's unit: 32 rows x 64 columns
}  // namespace wres

template <int C, int NW, int PD>
__global__ void __launch_bounds__(NW * 64, 1) conv_wres_kernel(const ConvArgs a) {
#pragma clang fp contract(off)
  using namespace wres;
  constexpr int NKT = 9 * C / BK;         // K-tiles
  constexpr int NCH = C / BK;             // 32-channel chunks
  constexpr int NPIECE = NKT * STAGE / 1024;
  static_assert(C % BK == 0 && NKT * STAGE <= 150 * 1024, "whole weight image in LDS");
  static_assert(PD == 1 || PD == 2, "A prefetch depth");
  __shared__ __attribute__((aligned(16))) unsigned char smem[NKT * STAGE];

  auto swzB = [](int R) { return ((R >> 2) & 3) ^ ((((R & 15) + 4) >> 3) & 1); };
  // weight column of K-tile t (the strip kernel's order)
  auto kcol = [](int t) {
    const int s = t / 3, kw = t - 3 * (t / 3);
    const int kh = s / NCH, ch = s - kh * NCH;
    return (kh * 3 + kw) * C + ch * BK;
  };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, g = lane >> 4;
  const ConvSeg& sg = a.seg[0];
  const int H = sg.H, W = sg.W, M = a.M, P = a.OH * a.OW;

  // ---- prologue: the whole split weight image, piece e = wave + NW j (stage e / 8) ----
  {
    const unsigned term_bytes = (unsigned)BN * (unsigned)a.Kpad * 2u;
    const __amdgpu_buffer_rsrc_t rsw =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.wh), (short)0, (int)(2 * term_bytes), 0x00020000);
    const int wlane = ((lane / 4) * a.Kpad + 8 * ((lane % 4) ^ swzB(lane / 4))) << 1;
    for (int e = wave; e < NPIECE; e += NW) {
      const int t = e >> 3, q = e & 7;  // stage t, piece q: term q / 4, rows 16 (q % 4) ..
      const unsigned off = (unsigned)(wlane + (int)((q >> 2) * term_bytes) + (q & 3) * 16 * a.Kpad * 2 + 2 * kcol(t));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(smem + e * 1024), 16,
                                               off, 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- this wave's units: XCD x owns units [U x / 8, U (x + 1) / 8), its waves take them in turn ----
  const int U = (M + WM - 1) / WM;
  const int xcd = blockIdx.x & 7, nbx = gridDim.x >> 3;
  const int u_lo = (int)((long long)U * xcd / 8), u_hi = (int)((long long)U * (xcd + 1) / 8);
  const int ustep = nbx * NW;
  int u = u_lo + (int)(blockIdx.x >> 3) * NW + wave;

  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(sg.x), (short)0, (int)sg.bytes, 0x00020000);
  // per unit and 16-row sub-tile: tap validity bits, the byte offset of (y - 1, x - 1) + the lane's
  // channel group, the frame's scale
  struct Rows {
    unsigned vmask[TM];
    int abase[TM];
    float as[TM];
  };
  auto setup = [&](int uu, Rows& r) {
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = uu * WM + mi * 16 + c16;
      const bool ok = m < M;
      const int mm = ok ? m : M - 1;
      const int x = mm % W, t = mm / W;
      const int y = t % H, b = t / H;
      unsigned msk = 0;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          if (ok && (unsigned)(y + kh - 1) < (unsigned)H && (unsigned)(x + kw - 1) < (unsigned)W)
            msk |= 1u << (kh * 3 + kw);
      r.vmask[mi] = msk;
      r.abase[mi] = ((((b * H + y - 1) * W + x - 1) * C) + 8 * g) * 4;
      float sinv;
      r.as[mi] = amax_frame_scale(a.amax_in, 1, mm / P, sinv);
    }
  };
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 raw[PD][TM][2];
  auto load_a = [&](const Rows& r, int t, u32x4 (&dst)[TM][2]) {
    const int s = t / 3, kw = t - 3 * (t / 3);
    const int kh = s / NCH, ch = s - kh * NCH;
    const int tap = kh * 3 + kw;
    const int toff = ((kh * W + kw) * C + ch * BK) * 4;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const bool ok = (r.vmask[mi] >> tap) & 1u;
      const unsigned off = ok ? (unsigned)(r.abase[mi] + toff) : 0x80000000u;
      dst[mi][0] = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
      dst[mi][1] = __builtin_amdgcn_raw_buffer_load_b128(rsx, off + 16u, 0, 0);
    }
  };
  const int bfo = c16 * BROW + ((g ^ swzB(c16)) << 4);  // this lane's W fragment in a block

  Rows cur, nxt;
  if (u < u_hi) {
    setup(u, cur);
#pragma unroll
    for (int p = 0; p < PD; ++p) load_a(cur, p, raw[p]);
  }
  for (; u < u_hi; u += ustep) {
    const int un = u + ustep;
    const bool more = un < u_hi;
    if (more) setup(un, nxt);
    f32x4_t acc[TM][TN];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    x6_f32x4 rv[TM][TN];
#pragma unroll
    for (int t = 0; t < NKT; ++t) {
      f16x8_t hf[2][TM];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
        split2h_x8(__builtin_bit_cast(x6_f32x4, raw[t % PD][mi][0]), __builtin_bit_cast(x6_f32x4, raw[t % PD][mi][1]),
                   cur.as[mi], hf[0][mi], hf[1][mi]);
      if (t + PD < NKT)
        load_a(cur, t + PD, raw[t % PD]);
      else if (more)
        load_a(nxt, t + PD - NKT, raw[t % PD]);  // the next unit's first K-tiles
      if (t == NKT - 3 && a.res) r3t_res_load<TM, TN>(a, rv, u * WM, 0, lane);
      const unsigned char* S = smem + t * STAGE + bfo;
      f16x8_t bq[TN][2];
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        bq[ni][0] = *reinterpret_cast<const f16x8_t*>(S + ni * 16 * BROW);
        bq[ni][1] = *reinterpret_cast<const f16x8_t*>(S + TERM_B + ni * 16 * BROW);
      }
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          f32x4_t cc = acc[mi][ni];
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(bq[ni][0], hf[1][mi], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(bq[ni][1], hf[0][mi], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(bq[ni][0], hf[0][mi], cc, 0, 0, 0);
          acc[mi][ni] = cc;
        }
      __builtin_amdgcn_sched_barrier(0);  // keep each K-tile's fragment reads in their K-tile
    }
    // ---- epilogue (r3t_epilogue_std's arithmetic, transposed accumulators: lane = 4 channels of
    // one row), frame maxima committed by this wave ----
    {
      const int mrow0 = u * WM;
      AmaxRows am(P, mrow0);
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int n = ni * 16 + 4 * g;
        const x6_f32x4 cs = *reinterpret_cast<const x6_f32x4*>(a.winv + n);
        const x6_f32x4 bn = a.bias ? *reinterpret_cast<const x6_f32x4*>(a.bias + n) : x6_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          const int m = mrow0 + mi * 16 + c16;
          const float ainv = 1.f / cur.as[mi];
          x6_f32x4 val;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            float tt = fmaf(acc[mi][ni][v] * ainv, cs[v], bn[v]);
            if (a.res) tt += rv[mi][ni][v];
            if (a.relu) tt = fmaxf(tt, 0.f);
            val[v] = tt;
          }
          if (m < M) {
            *reinterpret_cast<x6_f32x4*>(a.y + (size_t)m * BN + n) = val;
            if (a.amax_out)
              am.add(a.amax_out, m, fmaxf(fmaxf(fabsf(val[0]), fabsf(val[1])), fmaxf(fabsf(val[2]), fabsf(val[3]))));
          }
        }
      }
      if (a.amax_out) {
        float mx0 = am.mx0, mx1 = am.mx1;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
          mx0 = fmaxf(mx0, __shfl_xor(mx0, o, 64));
          mx1 = fmaxf(mx1, __shfl_xor(mx1, o, 64));
        }
        if (lane == 0) {
          if (mx0 > 0.f) amax_atomic(a.amax_out, am.fb0, mx0);
          if (mx1 > 0.f) amax_atomic(a.amax_out, am.fb0 + 1, mx1);
        }
      }
    }
    if (more) cur = nxt;
  }
}

// Launch-time checks (the kernel never bounds-checks these): one 3x3 / s1 / p1 segment with C
// input channels, N = 64, K = 9 C unsliced, no split-K, no upsampled residual.
template <int C, int NW, int PD>
inline int launch_conv_wres_cfg(const ConvArgs& a, hipStream_t st) {
  const ConvSeg& g = a.seg[0];
  if (!a.wh || !a.winv || a.nseg != 1 || g.KH != 3 || g.KW != 3 || g.stride != 1 || g.pad != 1 || g.C != C ||
      a.Kpad != 9 * C || a.N != wres::BN || a.OH != g.H || a.OW != g.W || a.wstride || a.wk0 || a.res_up ||
      a.ksplit > 1) {
    set_error("conv_wres: not a one-segment 3x3/s1/p1 conv with C=%d, N=64 (C=%d Kpad=%d N=%d)", C, g.C, a.Kpad,
              a.N);
    return SFA_E_UNSUPPORTED;
  }
  if ((long long)a.M * C * 4 >= (1ll << 31)) {
    set_error("conv_wres: input too large for 32-bit offsets");
    return SFA_E_UNSUPPORTED;
  }
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  // one block per CU (the weight image fills the LDS), a multiple of 8 (the XCD split), no more
  // blocks than the units need
  const int units = (a.M + wres::WM - 1) / wres::WM;
  int nblk = ncu & ~7;
  const int need = ((units + NW - 1) / NW + 7) & ~7;
  if (nblk > need) nblk = need;
  if (nblk < 8) nblk = 8;
  hipLaunchKernelGGL((conv_wres_kernel<C, NW, PD>), dim3((unsigned)nblk), dim3(NW * 64), 0, st, a);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

}  // namespace sfa
