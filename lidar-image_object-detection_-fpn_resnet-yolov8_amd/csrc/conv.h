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

enum ConvEpilogue { EPI_STD = 0, EPI_HEAD = 1 };

struct ConvArgs {
  ConvSeg seg[2];
  int nseg;
  int kseg1;           // first K index of segment 1 (multiple of 16)
  int Kpad;            // total K (multiple of 16)
  const float* w;      // [N][Kpad] (OHWI per segment, K-concatenated, zero padded)
  const uint16_t* wx;  // bf16x6 path: w split into 3 bf16 terms, [3][N][Kpad]
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
};

int launch_conv(const ConvArgs& a, int epilogue, int math, hipStream_t stream);

}  // namespace sfa
