// Implicit-GEMM convolution kernel template on fp32 MFMA for gfx950 (CDNA4).
//
// Every convolution of the KFPN forward (models/fpn_resnet.py:37-145, 53 convs,
// 62.57 GFLOP/frame) runs here as C[M][N] = A[M][K] * W[N][K]^T with
//   M = B*OH*OW output pixels (NHWC rows), N = Cout, K = taps*Cin (+ a 2nd segment).
// The A tile is gathered straight from the NHWC activation (no im2col buffer);
// BatchNorm is folded into W / bias on the host; bias, residual add and ReLU
// are fused into the epilogue; a downsample 1x1 conv is fused as a second
// K-segment; the detection heads' 1x1 convs run in the EPI_HEAD epilogue.
//
// MFMA: v_mfma_f32_32x32x2_f32 (exact f32 FMA chain, 64 FLOP/clk/SIMD — the
// fp32 matrix peak, 157.3 TF).  Lane l = (r = l&31, h = l>>5) feeds A[row r]
// and B[col r] at k-slot h; at k-step s the slot-h lanes carry actual k =
// (BK/2)h + s, so each lane reads BK/2 contiguous k of its row with ds_read_b128
// for a whole BK tile.  LDS rows are padded by 4 floats: BK = 16 (80-B rows) and
// BK = 32 (144-B rows) both put any 16 consecutive rows on 16 distinct 16-B bank
// groups, so the fragment reads are conflict-free.
#pragma once

#include "conv.h"

namespace sfa {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// GLDS: stage the A/B tiles with buffer_load ... lds (LDS-DMA, no VGPR staging)
//   into a 3-deep ring of unpadded, XOR-swizzled tiles (BK = 16 only).
// ABL: diagnostic ablation bits for tools/convbench (0 in the product):
//   1 = no global loads in the K loop, 2 = no barrier, 4 = no LDS fragment reads.
template <int BM, int BN, int WM, int WN, int BK, int EPI, int OCC, bool GLDS = false, int ABL = 0>
__global__ void __launch_bounds__(256, OCC) conv_mfma_kernel(const ConvArgs a) {
  static_assert(!GLDS || BK == 16, "the LDS-DMA ring is built for BK = 16");
  // GLDS rows are 64 B, quad q of row R stored at position q ^ ((R >> 2) & 3)
  constexpr int LDK = GLDS ? BK : BK + 4;
  constexpr int NSTAGE = GLDS ? 3 : 2;
  constexpr int WAVES_N = BN / WN;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per block");
  static_assert(BK == 16 || BK == 32, "BK");
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int QPR = BK / 4;         // float4 quads per tile row
  constexpr int RPP = 256 / QPR;      // rows covered per loader pass
  constexpr int A_LD = BM / RPP, B_LD = BN / RPP;
  static_assert(A_LD >= 1 && B_LD >= 1, "tile too small for the loader");
  constexpr int FR = BK / 8;          // float4 per fragment (BK/2 floats)
  constexpr int KS = BK / 2;          // k-steps per tile
  constexpr int STAGE = (BM + BN) * LDK;
  constexpr int HCH = BM < 128 ? BM : 128;  // head epilogue row chunk
  constexpr int HEAD_LDS = EPI == EPI_HEAD ? HCH * 65 : 0;
  constexpr int LDS_FLOATS = (NSTAGE * STAGE > HEAD_LDS) ? NSTAGE * STAGE : HEAD_LDS;
  __shared__ __attribute__((aligned(16))) float smem[LDS_FLOATS];
  float* lds_stage = smem;  // GLDS: destination stage of the next load_tile

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int n_tiles = a.N / BN;
  const int lbid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lbid / n_tiles, nt = lbid - mt * n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int M = a.M;

  // ---- loader geometry: thread -> (rows rr + RPP*i, k-quad kq).  Per row and
  // segment: the window origin (ihb, iwb) and its pixel index; per K-tile only the
  // tap offset is added.  Addresses are 32-bit byte offsets into a buffer
  // resource: an out-of-window tap gets an offset past the end and the hardware
  // returns zeros (the conv's zero padding) — no branch, no 64-bit math.
  // register mode: thread loads quad kq of row rr (+RPP*i); GLDS mode: lane l of wave
  // w fills row (w + 4i)*16 + (l >> 2) -- the same rows -- at LDS quad l & 3, which
  // holds logical quad (l & 3) ^ ((l >> 4) & 3)
  const int kq = GLDS ? ((lane & 3) ^ ((lane >> 4) & 3)) : tid % QPR;
  const int rr = tid / QPR;
  constexpr int NSEG = 2;
  int r_ih[NSEG][A_LD], r_iw[NSEG][A_LD], r_pix[NSEG][A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int m = m0 + rr + RPP * i;
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
      // rows past M: push the window out of range so every tap reads zeros
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
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.w), (short)0, (int)((unsigned)a.N * (unsigned)a.Kpad * 4u), 0x00020000);

  f32x4 ra[A_LD], rb[B_LD];
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
      // bitwise '&' (not '&&'): keeps this a select instead of divergent branches
      const bool ok = tap_ok & ((unsigned)(r_ih[sg][i] + kh) < (unsigned)g.H) &
                      ((unsigned)(r_iw[sg][i] + kw) < (unsigned)g.W);
      const unsigned off = ok ? (unsigned)((((r_pix[sg][i] + toff) << g.logC) + c) << 2) : 0x80000000u;
      if constexpr (GLDS) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(lds_stage + (wave + 4 * i) * 16 * BK), 16,
            off, 0, 0, 0);
      } else {
        ra[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      }
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
      const unsigned off = (unsigned)(((n0 + rr + RPP * j) * a.Kpad + k0 + 4 * kq) << 2);
      if constexpr (GLDS) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsw, (__attribute__((address_space(3))) void*)(lds_stage + (BM + (wave + 4 * j) * 16) * BK),
            16, off, 0, 0, 0);
      } else {
        rb[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsw, off, 0, 0));
      }
    }
  };
  auto store_tile = [&](int stage) {
    float* As = smem + stage * STAGE;
    float* Bs = As + BM * LDK;
#pragma unroll
    for (int i = 0; i < A_LD; ++i)
      *reinterpret_cast<f32x4*>(As + (rr + RPP * i) * LDK + 4 * kq) = ra[i];
#pragma unroll
    for (int j = 0; j < B_LD; ++j)
      *reinterpret_cast<f32x4*>(Bs + (rr + RPP * j) * LDK + 4 * kq) = rb[j];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[mi][ni][v] = 0.f;

  const int r = lane & 31, h = lane >> 5;
  auto compute = [&](int stage) {
    const float* As = smem + (ABL & 4 ? 0 : stage * STAGE);
    const float* Bs = As + BM * LDK;
    f32x4 af[TM][FR], bf[TN][FR];
    // row R = 32-row group base + r; with GLDS, (R >> 2) & 3 == (r >> 2) & 3
    const int sw = GLDS ? ((r >> 2) & 3) : 0;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const float* p = As + (wm * WM + mi * 32 + r) * LDK;
#pragma unroll
      for (int f = 0; f < FR; ++f)
        af[mi][f] = *reinterpret_cast<const f32x4*>(p + 4 * ((KS / 4 * h + f) ^ sw));
    }
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const float* p = Bs + (wn * WN + ni * 32 + r) * LDK;
#pragma unroll
      for (int f = 0; f < FR; ++f)
        bf[ni][f] = *reinterpret_cast<const f32x4*>(p + 4 * ((KS / 4 * h + f) ^ sw));
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const float av = af[mi][s >> 2][s & 3];
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const float bv = bf[ni][s >> 2][s & 3];
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[mi][ni], 0, 0, 0);
        }
      }
    }
  };

  const int nk = a.Kpad / BK;
  if constexpr (GLDS) {
    // 3-deep LDS-DMA ring: tiles kt+1 and kt+2 stream in while kt is consumed.
    constexpr int L = A_LD + B_LD;  // DMA instructions per wave per tile
    lds_stage = smem;
    load_tile(0);
    lds_stage = smem + STAGE;
    load_tile(nk > 1 ? 1 : 0);
    for (int kt = 0; kt < nk; ++kt) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");  // tile kt landed (this wave)
      __builtin_amdgcn_s_barrier();                              // ... and for every wave
      lds_stage = smem + ((kt + 2) % 3) * STAGE;                 // read last in iteration kt-1
      load_tile(kt + 2 < nk ? kt + 2 : nk - 1);
      compute(kt % 3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // Unconditional prefetch (the last iteration re-stages the final tile into the
    // idle buffer): keeps ra/rb in registers — a conditional definition made hipcc
    // spill them to scratch.
    if constexpr (!(ABL & 1)) load_tile(kt + 1 < nk ? kt + 1 : kt);
    compute(cur);
    store_tile(cur ^ 1);
    if constexpr (!(ABL & 2)) __syncthreads();
  }
  }

  if constexpr (EPI == EPI_STD) {
    AmaxRows am(a.OH * a.OW, m0);
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int n = n0 + wn * WN + ni * 32 + r;
      const float bn = a.bias[n];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int m = m0 + wm * WM + mi * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
          if (m < M) {
            float val = acc[mi][ni][v] + bn;
            if (a.res) val += a.res[(size_t)m * a.N + n];
            if (a.relu) val = fmaxf(val, 0.f);
            a.y[(size_t)m * a.N + n] = val;
            if (a.amax_out) am.add(a.amax_out, m, val);
          }
        }
      }
    }
    // consumers on the fp16x3 path scale by this (conv.h); the K loop's last barrier
    // retired every LDS read
    if (a.amax_out) amax_commit_block<4>(a.amax_out, am.fb0, am.mx0, am.mx1, smem);
  } else {
    // Detection head: ReLU(conv3x3 + b) staged in LDS (HCH rows at a time), then
    // the head's 1x1 conv (64 -> c <= 4) with bias, written channel-planar.
    static_assert(BN == 64, "one head (head_conv = 64 channels) per block column");
    float* T = smem;  // [HCH][65]; the K-loop's final barrier retired every LDS read
    int ch = 0, hoff = 0;
#pragma unroll
    for (int j = 0; j < SFA_MAX_HEADS; ++j)
      if (j == nt) {
        ch = a.hch[j];
        hoff = a.hoff[j];
      }
#pragma unroll
    for (int c0 = 0; c0 < BM; c0 += HCH) {
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int col = wn * WN + ni * 32 + r;
        const float bn = a.bias[n0 + col];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int row = wm * WM + mi * 32 + (v & 3) + 8 * (v >> 2) + 4 * h - c0;
            if (row >= 0 && row < HCH) T[row * 65 + col] = fmaxf(acc[mi][ni][v] + bn, 0.f);
          }
      }
      __syncthreads();
      for (int idx = tid; idx < HCH * ch; idx += 256) {
        const int row = idx % HCH, c = idx / HCH;
        const int m = m0 + c0 + row;
        if (m >= M) continue;
        const float* wr = a.hw1 + (nt * 4 + c) * 64;
        float s = a.hb1[nt * 4 + c];
        const float* tr = T + row * 65;
#pragma unroll 16
        for (int k = 0; k < 64; ++k) s = fmaf(tr[k], wr[k], s);
        a.hout[(size_t)(hoff + c) * M + m] = s;
      }
      __syncthreads();
    }
  }
}

template <int BM, int BN, int WM, int WN, int BK, int EPI, int OCC, bool GLDS = false, int ABL = 0>
inline int launch_conv_cfg(const ConvArgs& a, hipStream_t st) {
  if (a.Kpad % BK != 0 || (a.nseg == 2 && a.kseg1 % BK != 0) || a.N % BN != 0) {
    set_error("conv: K/N not aligned to the tile (Kpad=%d kseg1=%d N=%d, BK=%d BN=%d)", a.Kpad,
              a.kseg1, a.N, BK, BN);
    return SFA_E_UNSUPPORTED;
  }
  const int mt = ceil_div(a.M, BM);
  const int nt = a.N / BN;
  const long long nblocks = (long long)mt * nt;
  if (nblocks <= 0 || nblocks > 0x7fffffffll) {
    set_error("conv: bad grid (M=%d N=%d)", a.M, a.N);
    return SFA_E_INVALID;
  }
  hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, WN, BK, EPI, OCC, GLDS, ABL>), dim3((unsigned)nblocks),
                     dim3(256), 0, st, a);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

}  // namespace sfa
