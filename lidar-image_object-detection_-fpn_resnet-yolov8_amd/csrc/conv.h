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
};

enum ConvEpilogue { EPI_STD = 0, EPI_HEAD = 1 };

struct ConvArgs {
  ConvSeg seg[2];
  int nseg;
  int kseg1;           // first K index of segment 1 (multiple of 16)
  int Kpad;            // total K (multiple of 16)
  const float* w;      // [N][Kpad] (OHWI per segment, K-concatenated, zero padded)
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

int launch_conv(const ConvArgs& a, int epilogue, hipStream_t stream);

}  // namespace sfa
