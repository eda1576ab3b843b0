// 64 -> 64 3x3 / stride-1 / pad-1 convolution (the layer1 BasicBlock convs, fpn_resnet.py:42-71 at
// 152 x 152), fp16x3, WEIGHT-STATIONARY in VGPRs over full-width output rows (round 4).
//
// The strip kernel (conv_h3s_kernel.h) re-stages its W K-tile into LDS every k-step by LDS-DMA
// (8 KB per 128 output rows, one block-wide barrier per k-step: the round-3 ablations put the W
// staging at 10-16 % of the layer1 convs).  With K = 576 and 16 output channels per wave, a wave's
// whole weight slice in fp16x3 form is 576 x 16 x 2 terms x 2 B / 64 lanes = 144 VGPRs: here every
// wave loads it ONCE and keeps it for the whole launch, so the K loop has no W traffic and no
// barrier at all.
//
// Work.  A block owns output rows [y0, y1) of one frame (a segment; frames x segments blocks, about
// one per CU) and walks them one FULL image row at a time.  8 waves: wave w computes output channels
// 16 (w & 3) .. + 15 for the pixels [16 RB (w >> 2), 16 RB (w >> 2) + 16 RB) of the row (RB row
// blocks of 16 pixels; pixels >= W are computed on zero input and not stored).
//
// Input.  An LDS ring of 3 input rows (y - 1, y, y + 1), each split ONCE into its fp16 hi / lo terms at
// the frame's scale (every tap of the 9 reads the same split values; the strip kernel splits each
// input row once per kh), as 64-B rows of 32 channels per (row, chunk, term) with position p = x + 1
// (p = 0 and p > W hold zeros: the conv padding) and the strip kernel's pre-split swizzle (swzP:
// conflict-free ds_read_b128 at every kw offset).  After a row's K loop the ring slot of row y - 1
// takes row y + 2, whose loads were issued one row earlier; the residual tile of the next row is
// loaded the same way, so neither waits in the epilogue.
//
// Bits.  K order (kh, 32-channel chunk, kw), the three products per k-step (w_hi a_lo, w_lo a_hi,
// w_hi a_hi) on the transposed accumulators, the split (split2h_pair at the frame's scale) and the
// epilogue's rounding sequence are the strip kernel's: the outputs were bit-identical to
// conv_h3s_kernel<..., H3S_64> on the GPU (96², 160 x 192, 16 x 608², 5 x 608²).
//
// ROUND-4 EXPERIMENT, NOT ADOPTED (tools/convbench4 hook only): 134-137 us against the strip kernel's
// 121-124 in isolation, 116.8 vs ~102 us inside the forward, bench -1.4 % (profiles/r04e_*). At 243
// VGPRs (the 144-VGPR weight slice) hipcc keeps ONE A-fragment pair in flight and waits
// lgkmcnt(0) before every 3-MFMA group, so the LDS latency is exposed; a one-wave-per-SIMD form (4 waves
// x whole rows, accumulators in AGPRs) schedules the same way, and explicit double buffering spills.
#pragma once

#include "../../../lidar-image_object-detection_-fpn_resnet-yolov8_amd/csrc/conv_r3_kernel.h"

namespace sfa {

namespace conv_ws {
constexpr int NT = 512, NW = 8, C = 64, NCH = 2, TAPS = 9, KT = NCH * TAPS;  // 18 k-steps of 32
// widest row per instance (RB row blocks of 16 pixels per half): the 152-wide layer1 of a 608 input
// for RB = 5 (LDS: the ring and the staging row of W = 160 would not fit), else 32 RB
__host__ __device__ constexpr int wmax(int RB) { return RB == 5 ? 152 : 32 * RB; }
__host__ __device__ constexpr int npos(int RB) { return wmax(RB) + 2; }  // positions x = -1 .. W
__host__ __device__ constexpr int ring_bytes(int RB) { return 3 * NCH * 2 * npos(RB) * 64; }
__host__ __device__ constexpr int stage_bytes(int RB) { return wmax(RB) * C * 4; }
}  // namespace conv_ws

template <int RB>
__global__ void __launch_bounds__(512, 1) conv_ws_kernel(const ConvArgs a, int segs) {
#pragma clang fp contract(off)
  using namespace conv_ws;
  constexpr int NPOS = npos(RB), RROW = NPOS * 64;  // bytes of one (slot, chunk, term) row
  constexpr int RING = ring_bytes(RB), STAGE = stage_bytes(RB);
  constexpr int NI = (wmax(RB) * 16 + NT - 1) / NT;  // 16-B items (4 channels) of a row per thread
  constexpr int NPC = (STAGE / 1024 + NW - 1) / NW;  // 1-KiB staging DMA pieces per wave
  __shared__ __attribute__((aligned(16))) unsigned char smem[RING + STAGE + NW * 4];
  unsigned char* const stg = smem + RING;  // the next input row, f32 as in HBM (pixel-major, 64 ch)
  auto swzP = [](int R) { return ((R >> 2) & 1) << 1; };
  auto rowp = [&](int slot, int ch, int term) { return smem + ((slot * NCH + ch) * 2 + term) * RROW; };

  const ConvSeg& g = a.seg[0];
  const int H = g.H, W = g.W;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = wave & 3, half = wave >> 2;
  const int c16 = lane & 15, gq = lane >> 4;
  const int b = blockIdx.x / segs, sk = blockIdx.x - b * segs;
  const int y0 = sk * H / segs, y1 = (sk + 1) * H / segs;
  if (y1 <= y0) return;  // uniform per block

  // ---- this wave's weights: k-step t = (kh * NCH + chunk) * 3 + kw (the strip kernel's order) ----
  // lane (c16, gq) holds W[n = 16 cb + c16][k = K(t) + 8 gq .. + 7] of each term, K(t) = (kh 3 + kw) C + 32 chunk
  f16x8_t whi[KT], wlo[KT];
  {
    const size_t term = (size_t)a.N * a.Kpad;
    const uint16_t* wr = a.wh + (size_t)(16 * cb + c16) * a.Kpad + 8 * gq;
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const int kh = t / 6, ch = (t / 3) % 2, kw = t % 3;
      const int k0 = (kh * 3 + kw) * C + 32 * ch;
      whi[t] = *reinterpret_cast<const f16x8_t*>(wr + k0);
      wlo[t] = *reinterpret_cast<const f16x8_t*>(wr + term + k0);
    }
  }
  float ainv;
  const float sc = amax_frame_scale(a.amax_in, 1, b, ainv);

  // ---- ring: zero the padding positions (x = -1 and x = W) of every row once ----
  for (int i = tid; i < 3 * NCH * 2 * 2 * 4; i += NT) {
    const int q = i & 3, e = (i >> 2) & 1, row = i >> 3;
    *reinterpret_cast<x6_f32x4*>(smem + row * RROW + (e ? W + 1 : 0) * 64 + q * 16) = x6_f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // 16-B item i of an input row = pixel i >> 4, channels 4 (i & 15) .. + 3 (the HBM order)
  auto split_item = [&](int slot, int i, const x6_f32x4 v) {
    const int p = (i >> 4) + 1, cq = i & 15, ch = cq >> 3, q = cq & 7;
    const int off = p * 64 + (((q >> 1) ^ swzP(p)) << 4) + (q & 1) * 8;
    unsigned h0, h1, l0, l1;
    split2h_pair(v[0], v[1], sc, h0, l0);
    split2h_pair(v[2], v[3], sc, h1, l1);
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
    *reinterpret_cast<u32x2_t*>(rowp(slot, ch, 0) + off) = u32x2_t{h0, h1};
    *reinterpret_cast<u32x2_t*>(rowp(slot, ch, 1) + off) = u32x2_t{l0, l1};
  };
  const float* xf = g.x + (size_t)b * H * W * C;
  auto direct_row = [&](int yy) {  // load + split straight into the ring (the first rows of a segment)
    for (int i = tid; i < W * 16; i += NT) {
      x6_f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if ((unsigned)yy < (unsigned)H) v = *reinterpret_cast<const x6_f32x4*>(xf + ((size_t)yy * W + (i >> 4)) * C + 4 * (i & 15));
      split_item((yy + 3) % 3, i, v);
    }
  };
  // the next row into the staging area by LDS-DMA (1 KiB per wave instruction, rows outside the
  // image -> zeros through the buffer range)
  const __amdgpu_buffer_rsrc_t rsx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.x), (short)0, (int)g.bytes, 0x00020000);
  auto dma_row = [&](int yy) {
    const bool in = (unsigned)yy < (unsigned)H;
    const unsigned rbase = (unsigned)(((size_t)(b * H + yy) * W) * C * 4);
#pragma unroll
    for (int j = 0; j < NPC; ++j) {
      const int piece = wave + NW * j;
      if (piece * 1024 < W * C * 4) {
        const unsigned off = in && piece * 1024 + lane * 16 < W * C * 4 ? rbase + piece * 1024 + lane * 16 : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsx, (__attribute__((address_space(3))) void*)(stg + piece * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
  };
  auto stage_to_ring = [&](int yy) {
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = tid + k * NT;
      if (i < W * 16) split_item((yy + 3) % 3, i, *reinterpret_cast<const x6_f32x4*>(stg + i * 16));
    }
  };
  // residual tile of output row yy: lane (c16, gq) -> 4 channels of one pixel per row block
  const int xw0 = 16 * RB * half;
  auto load_res = [&](int yy, x6_f32x4 (&rv)[RB]) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int x = xw0 + 16 * rb + c16;
      rv[rb] = x6_f32x4{0.f, 0.f, 0.f, 0.f};
      if (a.res && x < W)
        rv[rb] = *reinterpret_cast<const x6_f32x4*>(a.res + ((size_t)(b * H + yy) * W + x) * a.N + 16 * cb + 4 * gq);
    }
  };

  for (int r = -1; r <= 1; ++r) direct_row(y0 + r);
  x6_f32x4 rv[RB];
  dma_row(y0 + 2);
  load_res(y0, rv);
  __syncthreads();

  float tmx = 0.f;  // this block's max |y| (its frame's amax)
  for (int y = y0; y < y1; ++y) {
    f32x4_t acc[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) acc[rb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const int kh = t / 6, ch = (t / 3) % 2, kw = t % 3;
      const unsigned char* rh = rowp((y + kh + 2) % 3, ch, 0);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int p = xw0 + 16 * rb + c16 + kw;  // position of input x = (output x) + kw - 1
        const int o = p * 64 + ((gq ^ swzP(p)) << 4);
        const f16x8_t ah = *reinterpret_cast<const f16x8_t*>(rh + o);
        const f16x8_t al = *reinterpret_cast<const f16x8_t*>(rh + RROW + o);
        f32x4_t cc = acc[rb];
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(whi[t], al, cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wlo[t], ah, cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(whi[t], ah, cc, 0, 0, 0);
        acc[rb] = cc;
      }
    }
    const bool more = y + 1 < y1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's staging pieces and residual loads
    __syncthreads();  // every wave is done with the slot of row y - 1; the staged row y + 2 landed
    if (more) stage_to_ring(y + 2);
    // epilogue of row y (r3t_epilogue_std's rounding sequence)
    {
      const x6_f32x4 cs = *reinterpret_cast<const x6_f32x4*>(a.winv + 16 * cb + 4 * gq);
      const x6_f32x4 bn = a.bias ? *reinterpret_cast<const x6_f32x4*>(a.bias + 16 * cb + 4 * gq) : x6_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int x = xw0 + 16 * rb + c16;
        x6_f32x4 val;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          float t = fmaf(acc[rb][v] * ainv, cs[v], bn[v]);
          if (a.res) t += rv[rb][v];
          if (a.relu) t = fmaxf(t, 0.f);
          val[v] = t;
        }
        if (x < W) {
          *reinterpret_cast<x6_f32x4*>(a.y + ((size_t)(b * H + y) * W + x) * a.N + 16 * cb + 4 * gq) = val;
          tmx = fmaxf(tmx, fmaxf(fmaxf(fabsf(val[0]), fabsf(val[1])), fmaxf(fabsf(val[2]), fabsf(val[3]))));
        }
      }
    }
    __syncthreads();  // row y + 2 is in the ring; the staging area is free
    if (more) {
      if (y + 2 < y1) dma_row(y + 3);
      load_res(y + 1, rv);
    }
  }
  if (a.amax_out) {
    float* red = reinterpret_cast<float*>(smem + RING + STAGE);
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

// One 64 -> 64 3x3/s1/p1 conv with the standard epilogue and no split-K, RB = ceil(W / 32) in {1, 2, 5}
// and W <= wmax(RB) (the layer1 widths of 96, 160 x 192 and 608 inputs); SFA_E_UNSUPPORTED otherwise.
inline int launch_conv_ws(const ConvArgs& a, hipStream_t st) {
  const ConvSeg& g = a.seg[0];
  if (!a.wh || !a.winv || a.nseg != 1 || g.C != conv_ws::C || a.N != 64 || g.KH != 3 || g.KW != 3 ||
      g.stride != 1 || g.pad != 1 || a.Kpad != 9 * conv_ws::C || a.OH != g.H || a.OW != g.W || a.ksplit > 1 ||
      a.res_up || a.wstride || a.wk0)
    return SFA_E_UNSUPPORTED;
  const int RB = (g.W + 31) / 32;
  if ((RB != 1 && RB != 2 && RB != 5) || g.W > conv_ws::wmax(RB)) return SFA_E_UNSUPPORTED;
  const int frames = a.M / (a.OH * a.OW);
  if (frames <= 0) return SFA_OK;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  int segs = (ncu + frames - 1) / frames;
  segs = segs < 1 ? 1 : (segs > g.H ? g.H : segs);
  const dim3 gd((unsigned)(frames * segs)), bd(conv_ws::NT);
  if (RB == 5)
    hipLaunchKernelGGL(conv_ws_kernel<5>, gd, bd, 0, st, a, segs);
  else if (RB == 2)
    hipLaunchKernelGGL(conv_ws_kernel<2>, gd, bd, 0, st, a, segs);
  else
    hipLaunchKernelGGL(conv_ws_kernel<1>, gd, bd, 0, st, a, segs);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

}  // namespace sfa
