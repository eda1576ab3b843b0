// Implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32) for gfx950.
#pragma once

#include "common.h"

namespace sfa {

// One K-segment of the implicit GEMM: an NHWC input read through a
// KHxKW/stride/pad window.  A conv with a fused 1x1 downsample residual, or an
// FPN 1x1 conv over a channel concat, is two segments concatenated along K.
struct ConvSeg {
  const float* x;
  int H, W, C, logC;   // C is a power of two (4 .. 512)
  int KH, KW, stride, pad;
  int taps;            // KH * KW
  int kdiv_mul, kdiv_sh;  // tap / KW == (tap * kdiv_mul) >> kdiv_sh for tap < 64
  unsigned bytes;      // size of x in bytes (< 2^31): buffer-load range, OOB -> 0
};

// Fills a segment; returns false if the tensor is too large for 32-bit offsets.
inline bool make_seg(ConvSeg& g, const float* x, int B, int H, int W, int C, int k, int stride, int pad) {
  g.x = x;
  g.H = H;
  g.W = W;
  g.C = C;
  g.logC = ilog2(C);
  g.KH = g.KW = k;
  g.stride = stride;
  g.pad = pad;
  g.taps = k * k;
  g.kdiv_mul = 1;
  g.kdiv_sh = 0;
  for (int sh = 0; sh < 16 && k > 1; ++sh) {
    const int mul = ((1 << sh) + k - 1) / k;
    bool ok = true;
    for (int t = 0; t < 64 && ok; ++t) ok = ((t * mul) >> sh) == t / k;
    if (ok) {
      g.kdiv_mul = mul;
      g.kdiv_sh = sh;
      break;
    }
  }
  const unsigned long long bytes = (unsigned long long)B * H * W * C * 4ull;
  g.bytes = (unsigned)bytes;
  return bytes < (1ull << 31);
}

// EPI_POOL (fp16x3 stem): bias + ReLU, then the 3x3/s2/p1 max-pool of the tile in LDS;
// y is the POOLED output (zeroed beforehand), rows of a block = one 16x16 spatial tile.
enum ConvEpilogue { EPI_STD = 0, EPI_HEAD = 1, EPI_POOL = 2 };

// fp16x3 activation scales (SFA_MATH_FP16X3).  max |x| of an activation tensor is kept
// PER FRAME (so a frame's result never depends on the rest of its batch), each in
// SFA_AMAX_WORDS words: SFA_AMAX_SHARDS shards one 128-B line apart, shard = blockIdx & 7
// of the producing workgroup; a reader takes the max over the shards.  Tensor t, frame b
// lives at base_t + b * SFA_AMAX_WORDS.
constexpr int SFA_AMAX_SHARDS = 8;
constexpr int SFA_AMAX_STRIDE = 32;   // words between shards
constexpr int SFA_AMAX_WORDS = SFA_AMAX_SHARDS * SFA_AMAX_STRIDE;

__device__ __forceinline__ void amax_atomic(unsigned* amax, int frame, float v) {
  atomicMax(amax + (size_t)frame * SFA_AMAX_WORDS + (blockIdx.x & (SFA_AMAX_SHARDS - 1)) * SFA_AMAX_STRIDE,
            __float_as_uint(v));
}

// Block-wide commit of the maxima of frames fb0 (mx0) and fb0 + 1 (mx1): every thread of
// the block calls it; one no-return atomic per frame and block.  `red` is 2 * NW floats of
// LDS no wave is using (the call synchronises the block).
template <int NW>
__device__ __forceinline__ void amax_commit_block(unsigned* amax, int fb0, float mx0, float mx1,
                                                  float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    mx0 = fmaxf(mx0, __shfl_xor(mx0, o, 64));
    mx1 = fmaxf(mx1, __shfl_xor(mx1, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    red[2 * (threadIdx.x >> 6)] = mx0;
    red[2 * (threadIdx.x >> 6) + 1] = mx1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float m0 = red[0], m1 = red[1];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      m0 = fmaxf(m0, red[2 * w]);
      m1 = fmaxf(m1, red[2 * w + 1]);
    }
    if (m0 > 0.f) amax_atomic(amax, fb0, m0);
    if (m1 > 0.f) amax_atomic(amax, fb0 + 1, m1);  // only rows of a real frame raise it
  }
}

// Scale of frame `frame` for an fp16x3 consumer: 2^(13 - e) for max |x| in [2^e, 2^(e+1))
// over its segments' inputs, so every scaled |x| < 2^14 (4x below the fp16 maximum);
// zero / unset / non-finite max -> 1.  sinv = 1 / s.
__device__ __forceinline__ float amax_frame_scale(const unsigned* const (&amax)[2], int nseg,
                                                  int frame, float& sinv) {
  unsigned mb = 0;
  for (int sg = 0; sg < nseg; ++sg)
    if (amax[sg]) {
      const unsigned* p = amax[sg] + (size_t)frame * SFA_AMAX_WORDS;
#pragma unroll
      for (int j = 0; j < SFA_AMAX_SHARDS; ++j) mb = max(mb, p[j * SFA_AMAX_STRIDE]);
    }
  if (mb == 0 || mb >= 0x7f800000u) {
    sinv = 1.f;
    return 1.f;
  }
  int e = (int)(mb >> 23) - 127;
  e = e < -100 ? -100 : (e > 100 ? 100 : e);
  sinv = __uint_as_float((unsigned)(127 - 13 + e) << 23);
  return __uint_as_float((unsigned)(127 + 13 - e) << 23);
}

// The same scale from the float bits of a max |x| (a tile's own maximum).
__device__ __forceinline__ float amax_scale_bits(unsigned mb, float& sinv) {
  if (mb == 0 || mb >= 0x7f800000u) {
    sinv = 1.f;
    return 1.f;
  }
  int e = (int)(mb >> 23) - 127;
  e = e < -100 ? -100 : (e > 100 ? 100 : e);
  sinv = __uint_as_float((unsigned)(127 - 13 + e) << 23);
  return __uint_as_float((unsigned)(127 + 13 - e) << 23);
}

// The scales of frames f0 and f1 (both < the batch's frame count) with all their words loaded before
// the first is reduced: one load round trip instead of two (round 5).
__device__ __forceinline__ void amax_frame_scale2(const unsigned* const (&amax)[2], int nseg, int f0, int f1,
                                                  float& s0, float& i0, float& s1, float& i1) {
  if (!amax[0]) {  // (not produced by this launcher: kept exact anyway)
    s0 = amax_frame_scale(amax, nseg, f0, i0);
    s1 = amax_frame_scale(amax, nseg, f1, i1);
    return;
  }
  const bool on1 = nseg > 1 && amax[1];
  const unsigned* p0 = amax[0] + (size_t)f0 * SFA_AMAX_WORDS;
  const unsigned* p1 = amax[0] + (size_t)f1 * SFA_AMAX_WORDS;
  unsigned w[2 * SFA_AMAX_SHARDS];
#pragma unroll
  for (int j = 0; j < SFA_AMAX_SHARDS; ++j) {
    w[j] = p0[j * SFA_AMAX_STRIDE];
    w[SFA_AMAX_SHARDS + j] = p1[j * SFA_AMAX_STRIDE];
  }
  if (on1) {
    const unsigned* q0 = amax[1] + (size_t)f0 * SFA_AMAX_WORDS;
    const unsigned* q1 = amax[1] + (size_t)f1 * SFA_AMAX_WORDS;
#pragma unroll
    for (int j = 0; j < SFA_AMAX_SHARDS; ++j) {
      w[j] = max(w[j], q0[j * SFA_AMAX_STRIDE]);
      w[SFA_AMAX_SHARDS + j] = max(w[SFA_AMAX_SHARDS + j], q1[j * SFA_AMAX_STRIDE]);
    }
  }
#pragma unroll
  for (int h = SFA_AMAX_SHARDS / 2; h >= 1; h >>= 1)
#pragma unroll
    for (int j = 0; j < h; ++j) {
      w[j] = max(w[j], w[j + h]);
      w[SFA_AMAX_SHARDS + j] = max(w[SFA_AMAX_SHARDS + j], w[SFA_AMAX_SHARDS + j + h]);
    }
  const unsigned mb0 = w[0], mb1 = w[SFA_AMAX_SHARDS];
  s0 = amax_scale_bits(mb0, i0);
  s1 = amax_scale_bits(mb1, i1);
}

enum StemInput { STEM_IN_NHWC4 = 0, STEM_IN_NCHW3 = 1, STEM_IN_NCHW3_FLIP = 2 };

// Producer side of a conv epilogue (rows m of the output, P = OH * OW rows per frame):
// frames fb0 and fb0 + 1 are reduced over the block, rows of later frames (blocks taller
// than a frame: small maps) are committed one by one.
struct AmaxRows {
  int P, fb0, mb1, mb2;
  float mx0 = 0.f, mx1 = 0.f;
  __device__ AmaxRows(int P_, int m0) : P(P_), fb0(m0 / P_), mb1((m0 / P_ + 1) * P_), mb2(mb1 + P_) {}
  __device__ __forceinline__ void add(unsigned* amax, int m, float val) {
    const float v = fabsf(val);
    if (m < mb1)
      mx0 = fmaxf(mx0, v);
    else if (m < mb2)
      mx1 = fmaxf(mx1, v);
    else if (v > 0.f)
      amax_atomic(amax, m / P, v);
  }
};

// n / d for 0 <= n < 2^31 by a multiply-high (round-up method with an add, Granlund-Montgomery):
// q = (umulhi(n, m) + n) >> s, s = ceil(log2 d), m = floor(2^32 (2^s - d) / d) + 1 < 2^32 — exact for
// every d >= 1 and n < 2^31 (the 33-bit magic 2^32 + m >= 2^(32+s) / d with an error below d <= 2^s).
// 3 VALU instead of the ~20 of a generic 32-bit division by a runtime divisor.
struct FastDiv {
  unsigned m;
  int s;
};
inline FastDiv make_fast_div(unsigned d) {
  int s = 0;
  while ((1ull << s) < d) ++s;
  const unsigned long long m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  return FastDiv{(unsigned)m, s};
}
__device__ __forceinline__ int fast_div(int n, FastDiv f) {
  return (int)((__umulhi((unsigned)n, f.m) + (unsigned)n) >> f.s);
}

struct ConvArgs {
  ConvSeg seg[2];
  int nseg;
  int kseg1;           // first K index of segment 1 (multiple of 16)
  int Kpad;            // total K (multiple of 16)
  const float* w;      // [N][Kpad] (OHWI per segment, K-concatenated, zero padded)
  const uint16_t* wx;  // bf16x6 path: w split into 3 bf16 terms, [3][N][Kpad]
  // fp16x3 path: w[n][k] * 2^e[n] split into 2 fp16 terms, [2][N][Kpad]; winv[n] = 2^-e[n]
  const uint16_t* wh;
  const float* winv;
  // fp16x3 path: per K-segment, the per-frame max |x| words of that segment's input
  // (written by its producer; frame b at + b * SFA_AMAX_WORDS), or null (scale 1)
  const unsigned* amax_in[2];
  unsigned* amax_out;  // this conv's per-frame max |y| is recorded here, or null
  const float* bias;   // [N]
  const float* res;    // residual [M][N] (NHWC) or nullptr
  float* y;            // output [M][N] (NHWC)
  int M, N, OH, OW;
  int relu;
  // EPI_HEAD: block column j = head j (64 channels each); bias+ReLU, then the
  // head's 1x1 conv (64 -> c_j <= 4) with bias, written channel-planar to
  // hout[(hoff[j] + c) * M + m].
  const float* hw1;    // [nheads][4][64]
  const float* hb1;    // [nheads][4]
  int hch[SFA_MAX_HEADS];
  int hoff[SFA_MAX_HEADS];
  float* hout;
  // split-K (EPI_STD, fp16x3): workspace for [ksplit][M][N] partial sums, or null (no
  // split); launch_conv picks ksplit for grids too small to fill the chip, the conv
  // writes scaled partials and a reduce kernel applies the epilogue.
  float* part;
  size_t part_floats;
  int ksplit;
  // fp16x3 (conv_h3_kernel) K-slice of a wider packed conv: the fp16 terms' row stride is
  // wstride (0: Kpad) and the slice starts at K column wk0. Used by the FPN 1x1 convs, which
  // run their two K-segments as two convs at different resolutions (model.hip).
  int wstride, wk0;
  // EPI_STD: residual given at HALF resolution [B][OH/2][OW/2][N], added bilinearly
  // upsampled x2 (align_corners, source step res_sh / res_sw), or null. bias may be null.
  const float* res_up;
  float res_sh, res_sw;
  // Round-3 experiment knobs (tools/experiments/r03 kernels and their convbench hooks only): tune
  // bits, stem ablations. The product kernels never read them and the model leaves them zero.
  int tune;
  int stem_abl;
  // split-K tickets (>= one word per output tile, zeroed before the launch): with them the last slice
  // of a tile combines the partials in the conv kernel (conv_h3_kernel.h splitk_ticket) instead of
  // splitk_reduce_kernel; null: the reduce launch
  unsigned* tile_cnt;
  int tile_cnt_words;  // capacity of tile_cnt (words): a launch with more output tiles takes the reduce launch
  // Patch stem input (stem_patch_kernel.h): STEM_IN_NHWC4 (the voxeliser's layout), STEM_IN_NCHW3
  // (the reference's (B, 3, H, W)), STEM_IN_NCHW3_FLIP (read as torch.flip(x, [2, 3])); every
  // 16 x 16 output tile scales its fp16x3 patch by its own max |x| (no layout / amax pass).
  int stem_in;
  // FPN 1x1 convs: 1 = may run on the persistent weight-resident kernel (fpn_kernel.h), 0 = the
  // per-tile conv_h3 / conv_r3 kernels (model option SFA_OPT_FPN_GEMM)
  int fpn_gemm;
  // multiply-high divisions by the input width / height (filled by the strip kernel's launch) and by
  // the output width / height (conv_r3's)
  FastDiv fd_w, fd_h, fd_ow, fd_oh;
};

// Bilinear x2 (align_corners) sample of a half-resolution NHWC tensor at output pixel
// (b, oh, ow), channel n — F.interpolate(scale_factor=2, mode='bilinear', align_corners=True)
// as upsample2x_bilinear_kernel evaluates it.
__device__ __forceinline__ float res_up_sample(const ConvArgs& a, int m, int n) {
  const int ow = m % a.OW, t = m / a.OW;
  const int oh = t % a.OH, b = t / a.OH;
  const int H = a.OH >> 1, W = a.OW >> 1;
  const float fy = a.res_sh * (float)oh, fx = a.res_sw * (float)ow;
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = y0 + (y0 < H - 1 ? 1 : 0), x1 = x0 + (x0 < W - 1 ? 1 : 0);
  const float ly1 = fy - (float)y0, lx1 = fx - (float)x0;
  const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
  const float* r = a.res_up + (size_t)b * H * W * a.N + n;
  const float a00 = r[(y0 * W + x0) * a.N], a01 = r[(y0 * W + x1) * a.N];
  const float a10 = r[(y1 * W + x0) * a.N], a11 = r[(y1 * W + x1) * a.N];
  return fmaf(ly0, fmaf(lx0, a00, lx1 * a01), ly1 * fmaf(lx0, a10, lx1 * a11));  // as r3t_epilogue_std
}

int launch_conv(const ConvArgs& a, int epilogue, int math, hipStream_t stream);
// fp16x3 stem 7x7/s2 + BN + ReLU + max-pool 3x3/s2 in one kernel over 16 x 16 patches + a merge
// pass (stem_patch_kernel.h); SFA_E_UNSUPPORTED if the stem's shape does not tile 16 x 16.
int launch_stem_patch(const ConvArgs& a, hipStream_t stream);

}  // namespace sfa
