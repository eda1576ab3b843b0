// Weight-stationary persistent implicit-GEMM convolution for the 64-wide layer1 convs
// (fpn_resnet.py BasicBlock conv1 / conv2 at 152x152, C = N = 64, 3x3, stride 1), fp16x3 on
// v_mfma_f32_16x16x32_f16 with f32 accumulation (gfx950 / CDNA4).
//
// Same GEMM view, operand split, frame scales, K order (chunk-major) and transposed accumulators
// as conv_r3_kernel (conv_r3_kernel.h); what differs is where the weights live and how the
// work is scheduled. The whole fp16 weight image (2 terms x 64 rows x Kpad: 144 KiB for
// K = 576) is copied into LDS ONCE per workgroup, and each CU runs one workgroup for the whole
// launch (grid = CUs): its waves walk a contiguous chunk of 32-row wave tiles (interleaved, so
// the 8 waves of a CU work on neighbouring rows and share the 3x3 halo in L1 / L2). A wave
// never waits for another wave after the weight copy: no per-K-tile DMA, no barrier; its A
// fragments (8 channels of one input pixel per lane, buffer loads straight into VGPRs, zero
// outside the image) are prefetched PF K-tiles ahead across tile boundaries, the W fragments
// are LDS reads one K-tile ahead, and the epilogue (bias, residual, ReLU, float4 NHWC stores,
// per-frame max) is per wave. For a 64-wide conv the round-2 strip kernel re-staged the
// weights for every 128-row block: 144 KiB per block, more than its A strip.
#pragma once

#include "conv_r3_kernel.h"

namespace sfa {

// NK: K-tiles of 32 (Kpad / 32); PF: A prefetch distance in K-tiles (NK % PF == 0, so the
// register ring slot of a K-tile is the same in every wave tile).
template <int WM, int NW, int NK, int PF, int ABL = 0>
__global__ void __launch_bounds__(NW * 64, 1) conv_ws_kernel(const ConvArgs a) {
#pragma clang fp contract(off)
  constexpr int BN = 64, TN = BN / 16, TM = WM / 16;
  constexpr int BK = 32, BROW = BK * 2;
  constexpr int TERM_B = BN * BROW, STAGE = 2 * TERM_B;  // per K-tile: 4 KiB per term
  constexpr int ND_BT = TERM_B / 1024, ND_B = 2 * ND_BT;  // 1-KiB DMA pieces per K-tile
  static_assert(NK % PF == 0 && PF >= 1 && PF <= 3, "A ring");
  static_assert(NK * STAGE + 2 * BN * 4 <= 160 * 1024, "weights must fit the LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[NK * STAGE + 2 * BN * 4];
  float* const s_winv = reinterpret_cast<float*>(smem + NK * STAGE);  // epilogue constants
  float* const s_bias = s_winv + BN;

  auto swzB = [](int R) { return ((R >> 2) & 3) ^ ((((R & 15) + 4) >> 3) & 1); };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, g = lane >> 4;
  const int M = a.M;
  const ConvSeg& sg0 = a.seg[0];

  // chunk-major K order: K-tile kt = tap kt % taps of the 32-channel chunk kt / taps
  auto kcol = [&](int kt) -> int {
    const int chunk = (kt * 7282) >> 16;  // kt / 9 (3x3, checked at launch)
    return (kt - 9 * chunk) * sg0.C + chunk * BK;
  };

  // ---- weights: every K-tile into its own LDS stage (the conv_r3 stage image) ----
  {
    const int wst = a.Kpad;
    const unsigned term_bytes = (unsigned)a.N * (unsigned)wst * 2u;
    const __amdgpu_buffer_rsrc_t rsw =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.wh), (short)0, (int)(2 * term_bytes), 0x00020000);
    const int wlane = (((lane / 4) * wst + 8 * ((lane % 4) ^ swzB(lane / 4))) << 1);
    for (int e = wave; e < NK * ND_B; e += NW) {
      const int kt = e / ND_B, p = e - kt * ND_B;
      const int boff = (int)((p / ND_BT) * term_bytes) + (p % ND_BT) * 16 * wst * 2 + 2 * kcol(kt);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsw, (__attribute__((address_space(3))) void*)(smem + kt * STAGE + p * 1024), 16, (unsigned)(wlane + boff), 0, 0,
          0);
    }
  }

  // ---- this workgroup's wave tiles: a contiguous chunk (neighbouring chunks on one XCD) ----
  const int T = (M + WM - 1) / WM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int per = (T + gridDim.x - 1) / gridDim.x;
  const int t_lo = bid * per, t_hi = min(T, t_lo + per);

  const __amdgpu_buffer_rsrc_t rs0 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(sg0.x), (short)0, (int)sg0.bytes, 0x00020000);
  // per tile: the tap-validity bits and the byte offset of each of the lane's rows
  struct Meta {
    unsigned vmask[TM], abase[TM];
  };
  auto setup = [&](Meta& mt, int t) {
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = t * WM + mi * 16 + c16;
      const bool ok = t < t_hi && m < M;
      const int mm = ok ? m : 0;
      const int ow = mm % a.OW, q = mm / a.OW;
      const int oh = q % a.OH, b = q / a.OH;
      const int ih = ok ? oh * sg0.stride - sg0.pad : -16384;
      const int iw = ow * sg0.stride - sg0.pad;
      unsigned msk = 0;
      for (int tp = 0; tp < sg0.taps; ++tp) {
        const int kh = (tp * sg0.kdiv_mul) >> sg0.kdiv_sh, kw = tp - kh * sg0.KW;
        if ((unsigned)(ih + kh) < (unsigned)sg0.H && (unsigned)(iw + kw) < (unsigned)sg0.W) msk |= 1u << tp;
      }
      mt.vmask[mi] = msk;
      mt.abase[mi] = (unsigned)(((((b * sg0.H + ih) * sg0.W + iw) << sg0.logC) + 8 * g) << 2);
    }
  };
  r3_u32x4 raw[PF][TM][2];
  auto load_a = [&](const Meta& mt, int kt, r3_u32x4 (&dst)[TM][2]) {
    const int k0 = kcol(kt);
    const int tap = k0 >> sg0.logC, c0 = k0 & (sg0.C - 1);
    const int kh = (tap * sg0.kdiv_mul) >> sg0.kdiv_sh, kw = tap - kh * sg0.KW;
    const unsigned toff = (unsigned)((((kh * sg0.W + kw) << sg0.logC) + c0) << 2);
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const bool ok = (mt.vmask[mi] >> tap) & 1u;
      const unsigned off = ok ? mt.abase[mi] + toff : 0x80000000u;
      dst[mi][0] = __builtin_amdgcn_raw_buffer_load_b128(rs0, off, 0, 0);
      dst[mi][1] = __builtin_amdgcn_raw_buffer_load_b128(rs0, off + 16u, 0, 0);
    }
  };
  // W fragments: block p = kt * TN + ni of a tile in ring slot p % RS, read RA blocks ahead
  constexpr int RA = 2, RS = RA + 1;
  static_assert((NK * TN) % RS == 0, "W ring slots must repeat per tile");
  const int bfo = c16 * BROW + ((g ^ swzB(c16)) << 4);
  f16x8_t wq[RS][2];
  auto read_w = [&](int p) {
    const unsigned char* S = smem + (p / TN) * STAGE + (p % TN) * 16 * BROW + bfo;
    wq[p % RS][0] = *reinterpret_cast<const f16x8_t*>(S);
    wq[p % RS][1] = *reinterpret_cast<const f16x8_t*>(S + TERM_B);
  };
  if (tid < BN) {
    s_winv[tid] = a.winv[tid];
    s_bias[tid] = a.bias ? a.bias[tid] : 0.f;
  }
  AmaxRows am(a.OH * a.OW, min(t_lo * WM, M - 1));

  Meta cur, nxt;
  int t = t_lo + wave;
  setup(cur, t);
  if (t < t_hi) {
#pragma unroll
    for (int s = 0; s < PF; ++s) load_a(cur, s, raw[s]);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PF * 2 * TM) : "memory");  // the weight copy has landed
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  for (; t < t_hi; t += NW) {
    const int tn = t + NW;
    setup(nxt, tn);  // rows past t_hi get no valid taps: their loads return zeros
    float as[TM], ainv[TM];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = min(t * WM + mi * 16 + c16, M - 1);
      float sinv;
      as[mi] = amax_frame_scale(a.amax_in, 1, m / (a.OH * a.OW), sinv);
      ainv[mi] = 1.f / as[mi];
    }
    f32x4_t acc[TM][TN];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < RA; ++p) read_w(p);
    x6_f32x4 rv[TM][TN];
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
      f16x8_t hf[2][TM];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
        split2h_x8(__builtin_bit_cast(x6_f32x4, raw[kt % PF][mi][0]), __builtin_bit_cast(x6_f32x4, raw[kt % PF][mi][1]),
                   as[mi], hf[0][mi], hf[1][mi]);
      const int s = kt + PF;  // the K-tile whose A is loaded now: this tile's or the next one's
      if (s < NK)
        load_a(cur, s, raw[s % PF]);
      else
        load_a(nxt, s - NK, raw[s % PF]);
      if (kt == NK - 2 && a.res) {  // the residual tile, ahead of the last K-tiles
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni) {
            const int m = min(t * WM + mi * 16 + c16, M - 1);
            rv[mi][ni] = *reinterpret_cast<const x6_f32x4*>(a.res + (size_t)m * a.N + ni * 16 + 4 * g);
          }
      }
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int p = kt * TN + ni;
        if (p + RA < NK * TN) read_w(p + RA);
        const f16x8_t c0 = wq[p % RS][0], c1 = wq[p % RS][1];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          f32x4_t cc = acc[mi][ni];
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[1][mi], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c1, hf[0][mi], cc, 0, 0, 0);
          cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(c0, hf[0][mi], cc, 0, 0, 0);
          acc[mi][ni] = cc;
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // keep each K-tile's loads and LDS reads in place
    }
    // epilogue (r3t_epilogue_std's arithmetic): lane = 4 channels of one row
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = t * WM + mi * 16 + c16;
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const x6_f32x4 cs = *reinterpret_cast<const x6_f32x4*>(s_winv + ni * 16 + 4 * g);
        const x6_f32x4 bn = *reinterpret_cast<const x6_f32x4*>(s_bias + ni * 16 + 4 * g);
        x6_f32x4 val;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          float r = fmaf(acc[mi][ni][v] * ainv[mi], cs[v], bn[v]);
          if (a.res) r += rv[mi][ni][v];
          if (a.relu) r = fmaxf(r, 0.f);
          val[v] = r;
        }
        if (m < M) {
          *reinterpret_cast<x6_f32x4*>(a.y + (size_t)m * a.N + ni * 16 + 4 * g) = val;
          if (a.amax_out)
            am.add(a.amax_out, m, fmaxf(fmaxf(fabsf(val[0]), fabsf(val[1])), fmaxf(fabsf(val[2]), fabsf(val[3]))));
        }
      }
    }
    cur = nxt;
  }
  if (a.amax_out) {  // this wave's maxima of the chunk's first two frames
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

template <int WM, int NW, int NK, int PF, int ABL = 0>
inline int launch_conv_ws_cfg(const ConvArgs& a, hipStream_t st, int ncu) {
  const ConvSeg& g = a.seg[0];
  if (!a.wh || !a.winv || a.nseg != 1 || a.N != 64 || g.taps != 9 || g.C < 32 || (g.C & (g.C - 1)) != 0 ||
      a.Kpad != 9 * g.C || a.Kpad != NK * 32 || a.wstride || a.wk0 || a.res_up || a.ksplit > 1) {
    set_error("conv_ws: needs one 3x3 segment, C a power of two >= 32, N = 64, Kpad = %d (C=%d N=%d Kpad=%d)", NK * 32,
              g.C, a.N, a.Kpad);
    return SFA_E_UNSUPPORTED;
  }
  if ((long long)a.M * a.N >= (1ll << 31) || ncu <= 0) {
    set_error("conv_ws: bad size (M=%d)", a.M);
    return SFA_E_INVALID;
  }
  const int T = ceil_div(a.M, WM);
  const int grid = T < ncu ? T : ncu;
  hipLaunchKernelGGL((conv_ws_kernel<WM, NW, NK, PF, ABL>), dim3((unsigned)grid), dim3(NW * 64), 0, st, a);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

}  // namespace sfa
