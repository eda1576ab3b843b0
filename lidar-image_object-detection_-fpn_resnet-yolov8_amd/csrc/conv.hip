// Convolution dispatch: picks the kernel (fp16x3, bf16x6 or f32 MFMA) and its tile
// configuration per layer shape (conv_*_kernel.h).
#include <cstdlib>

#include "conv_kernel.h"
#include "conv_x6_kernel.h"
#include "conv_h3_kernel.h"
#include "conv_h3s_kernel.h"
#include "conv_r3_kernel.h"
#include "fpn_kernel.h"
#include "stem_patch_kernel.h"

namespace sfa {

// Tile choices are priced at the bench batch (16 frames of the launch's geometry), never at
// a.M: different kernels sum in different orders, so a choice by the batch's row count would
// let a frame's result depend on the batch it is computed in (tests/test_gpu_model.py
// test_batch_invariance_608 holds every path to bit-identical frames across batches).
static long long tile_rows(const ConvArgs& a) { return 16LL * a.OH * a.OW; }

// bf16x6 tiles per shape, from tools/convbench.hip sweeps on MI355X (round 1):
// wide-N tiles amortise the A split; 8-wave LDS-DMA tiles for the big-M layers.
// Returns SFA_E_UNSUPPORTED when no bf16x6 tile fits (the caller falls back to f32).
static int launch_conv_x6(const ConvArgs& a, int epilogue, hipStream_t st) {
  if (!a.wx) return SFA_E_UNSUPPORTED;
  auto ok = [](int rc) { return rc != SFA_E_UNSUPPORTED; };
  int rc = SFA_E_UNSUPPORTED;
  if (epilogue == EPI_HEAD) {
    if (a.N == 320) rc = launch_conv_x6g_cfg<256, 320, 32, EPI_HEAD, 1>(a, st);
    if (!ok(rc)) rc = launch_conv_x6_cfg<128, 64, 32, 64, 32, EPI_HEAD, 2>(a, st);
    if (!ok(rc)) rc = launch_conv_x6g_cfg<256, 64, 32, EPI_HEAD, 1>(a, st);
    return rc;
  }
  if (a.N == 64) return launch_conv_x6g_cfg<256, 64, 32, EPI_STD, 1>(a, st);
  if (a.N % 128 == 0) {
    if (tile_rows(a) >= 50000) rc = launch_conv_x6_cfg<128, 128, 64, 64, 16, EPI_STD, 2>(a, st);
    else if (tile_rows(a) >= 10000) rc = launch_conv_x6g_cfg<128, 128, 32, EPI_STD, 2>(a, st);
    else rc = launch_conv_x6_cfg<64, 128, 32, 64, 32, EPI_STD, 2>(a, st);
    if (!ok(rc)) rc = launch_conv_x6g_cfg<128, 128, 32, EPI_STD, 2>(a, st);
  }
  return rc;
}

// Split-K slices of a 128 x 128-tiled body conv (fp16x3, standard epilogue with bias): 2 for the
// 512-wide (layer4) convs, whose 184 output tiles cannot fill 256 CUs (-13..16 %), combined by
// splitk_reduce_kernel. Chosen from the conv width only, so a frame's arithmetic never depends
// on its batch. (Balanced split counts with the slices combined in the kernel were measured 35 %
// slower: tools/experiments/r03, profiles/r03e_ab_splitk_inkernel.txt.)
static int pick_ksplit(const ConvArgs& a) {
  if (!a.part || !a.bias || a.wstride || a.wk0 || a.res_up) return 1;
  return a.N >= 512 ? 2 : 1;
}

// One-segment 3x3 / stride 1 / pad 1 conv with 32-channel chunks: conv_h3s_kernel applies.
static bool strip_ok(const ConvArgs& a) {
  const ConvSeg& g = a.seg[0];
  return a.nseg == 1 && g.KH == 3 && g.KW == 3 && g.stride == 1 && g.pad == 1 && g.C >= 32 &&
         (g.C & 31) == 0 && a.Kpad == 9 * g.C && a.OH == g.H && a.OW == g.W;
}

// fp16x3 kernels per shape (tools/convbench.hip sweeps). Round 4 keeps only
// the adopted kernels here; every measured-and-rejected variant (the round-2/3 SFA_TUNE bits) is in
// tools/experiments/r03/ with its convbench hook.
//  * heads: conv_r3_kernel 256 x 320 (all 5 heads of a level per tile), half-tile stagger, 3-stage
//    W ring, 3-block W read-ahead, scalar taps, chunk-major K order, packed head epilogue;
//  * 3x3/s1 body convs: conv_h3s_kernel (A staged once per kh as a row strip for the three kw
//    taps), transposed float4 epilogue, v_fma_mix split; 64-wide 128 x 64 at 3 blocks / CU with the
//    pre-split strip and the residual loaded during the last super-step, 128..512-wide 128 x 128
//    (split-K 2 for the 512-wide; the 256-wide layer3 convs on 64 x 128 tiles);
//  * big-M (layer2) stride-2 and conv + downsample convs: conv_r3_kernel 128 x 128 (A in registers,
//    chunk-major K), -25 % on layer2.0.conv1 against conv_h3;
//  * FPN skip convs (half-resolution residual added bilinearly upsampled in the epilogue):
//    conv_r3_kernel, float4 taps;
//  * the rest (layer3/4 stride-2 and conv + downsample, the FPN low-resolution 1x1 convs, the stem
//    without the patch kernel): conv_h3_kernel on 16x16x32 MFMAs.
// conv_r3_kernel ABL values (conv_r3_kernel.h bit list): 256 spread W DMA | 2048 transposed
// accumulators, always; 524288 chunk-major K order (the 3x3 window's 32-channel slices stay in L2
// across the 9 taps; heads' HBM traffic 3.5-4.7x lower: profiles/r02_convbench_cmaj.txt);
// 32768 the upsampled-residual epilogue (FPN skip convs).
constexpr int R3_BODY = 256 | 2048 | 524288;
constexpr int R3_FPN = 256 | 2048 | 32768;
// heads: + s_setprio 1 for waves 4-7 (4), v_fma_mix split (4096), 3-block W read-ahead (8192), scalar
// tap decode (16384), packed epilogue (65536), waves 4-7 half a K-tile behind their SIMD partners
// with three W stages (1048576: -4.6 / -3.1 / -1.0 % per launch on L1 / L2 / L0, bit-identical,
// profiles/r03h_convbench_heads_stagger.txt), the delayed half issuing every W DMA piece of the K loop
// (2097152, round 5: -2.2 %, bit-identical, profiles/r05ah_heads_delayed_half_dma.txt)
constexpr int R3_HEAD_STAG = 256 | 2048 | 4 | 4096 | 8192 | 16384 | 65536 | 524288 | 1048576 | 2097152;
// strip kernel (conv_h3s_kernel.h bits): transposed epilogue (2), v_fma_mix split (8), the pre-split
// strip (4) and the residual tile loaded during the last super-step (128) on every tile shape (round
// 5: with the one-latency presplit the 128-wide tiles gain from them too, layer2 -4.6 % / -6.5 % with a
// residual, layer3 -1 / -2 %, bit-identical: profiles/r05j_*; the names of the former two forms stay),
// the strip in registers instead of an LDS-DMA buffer (1024, late round 5: layer1 -2.7 %, layer2 -2.2 %,
// layer4 -2.8 %, bench +0.6 %, bit-identical, profiles/r05bi_*)
constexpr int H3S_64 = 2 | 4 | 8 | 128 | 1024;
constexpr int H3S_128 = 2 | 4 | 8 | 128 | 1024;
// 128 x 128 tiles (layer2): at 3 blocks / CU without the residual prefetch (198 -> 168 VGPRs; the strip in
// registers freed the LDS), 722 tiles in one round of 768 slots: -1.9 %, bit-identical, profiles/r05bj_*
constexpr int H3S_128W = 2 | 4 | 8 | 1024;

// FPN 1x1 convs (commuted: the low-resolution W_a . x and the skip conv with the upsampled
// residual) on the persistent weight-resident kernel (fpn_kernel.h), by channel count.
static int launch_fpn(const ConvArgs& a, hipStream_t st) {
  const int C = a.seg[0].C;
  if (a.res_up) {
    if (a.OW <= 2 * fpn_seg::WHMAX) {  // narrow levels: flat pixel steps, the taps from an LDS row ring
      const int rc = C == 128 ? launch_fpn_seg_cfg<128, 1>(a, st) : C == 256 ? launch_fpn_seg_cfg<256, 1>(a, st)
                                                                             : SFA_E_UNSUPPORTED;
      if (rc != SFA_E_UNSUPPORTED) return rc;
    }
    {  // full rows, the bilinear taps from an LDS ring of source rows
      const int rc = launch_fpn_row(a, st);
      if (rc != SFA_E_UNSUPPORTED) return rc;
    }
    if (C == 64 && a.N % 64 == 0) return launch_fpn_gemm_cfg<64, 64, true, 3>(a, st);
    if (C == 128 && a.N % 128 == 0) return launch_fpn_gemm_cfg<128, 128, true, 2>(a, st);
    if (C == 256 && a.N % 128 == 0) return launch_fpn_gemm_cfg<256, 128, true, 1>(a, st);
  } else {
    if (C == 128 && a.N % 64 == 0) return launch_fpn_gemm_cfg<128, 64, false, 4>(a, st);
    if (C == 256 && a.N % 128 == 0) return launch_fpn_gemm_cfg<256, 128, false, 1>(a, st);
    if (C == 512 && a.N % 64 == 0) return launch_fpn_gemm_cfg<512, 64, false, 1>(a, st);
  }
  return SFA_E_UNSUPPORTED;
}

static int launch_conv_h3(const ConvArgs& a, int epilogue, hipStream_t st) {
  if (!a.wh || !a.winv) return SFA_E_UNSUPPORTED;
  auto ok = [](int rc) { return rc != SFA_E_UNSUPPORTED; };
  int rc = SFA_E_UNSUPPORTED;
  const bool sliced = a.wstride || a.wk0 || a.res_up;  // conv_h3_kernel reads these; the others do not
  const bool strip = strip_ok(a) && !sliced;
  if (epilogue == EPI_HEAD) {
    if (a.N == 320) rc = launch_conv_r3_cfg<256, 320, 32, EPI_HEAD, 1, 3, R3_HEAD_STAG>(a, st);
    if (!ok(rc)) rc = launch_conv_x6g_cfg<256, 64, 32, EPI_HEAD, 1, 16, 3, 0, 64, 1>(a, st);  // other head counts
    return rc;
  }
  if (a.fpn_gemm && sliced && a.nseg == 1 && a.seg[0].KH == 1 && a.seg[0].KW == 1 && a.seg[0].stride == 1) {
    rc = launch_fpn(a, st);  // the FPN 1x1 convs (commuted)
    if (ok(rc)) return rc;
  }
  if (a.res_up) {  // FPN skip convs of other widths: conv_r3, transposed float4 epilogue, float4 taps
    if (a.N == 64)
      rc = launch_conv_r3_cfg<128, 64, 32, EPI_STD, 4, 2, R3_FPN>(a, st);
    else if (a.N % 128 == 0)
      rc = launch_conv_r3_cfg<128, 128, 32, EPI_STD, 2, 2, R3_FPN>(a, st);
    return rc;
  }
  if (a.N == 64) {
    if (strip) rc = launch_conv_h3s_cfg<128, 64, 32, EPI_STD, 3, H3S_64>(a, st);
    if (!ok(rc) && a.Kpad >= 256) rc = launch_conv_h3_cfg<256, 64, 32, EPI_STD, 1, 32, 2, false, 0, 1>(a, st);
    if (!ok(rc)) rc = launch_conv_h3_cfg<128, 64, 32, EPI_STD, 2, 16, 3, false, 0>(a, st);
    if (!ok(rc) && !sliced) rc = launch_conv_x6g_cfg<256, 64, 32, EPI_STD, 1, 16, 3, 0, 64, 1>(a, st);
    return rc;
  }
  if (a.N % 128 == 0) {
    ConvArgs b = a;
    b.ksplit = pick_ksplit(a);
    if (strip && b.ksplit == 1 && a.N == 256 && tile_rows(a) < 50000)
      // layer3 (362 128-row tiles for 512 block slots): 64 x 128 tiles at 3 blocks / CU fill the
      // chip; same per-element K order, so the same bits (tools/convbench4: 97.7 vs 102.0 us,
      // profiles/r04a_convbench4_stem_regw_tiles.txt)
      rc = launch_conv_h3s_cfg<64, 128, 16, EPI_STD, 3, H3S_128>(b, st);
    else if (strip && b.ksplit == 2 && a.N == 512 && tile_rows(a) < 50000)
      // layer4 (184 128 x 128 tiles x 2 slices for 512 block slots): the 64-wide layer1 form, 128 x 64
      // tiles at 3 blocks / CU (736 blocks for 768 slots); same slices and per-element K order, so the
      // same bits (tools/convbench4: 102.4-105.0 vs 107.4-110.7 us, profiles/r04o_convbench4_layer4_splits.txt)
      rc = launch_conv_h3s_cfg<128, 64, 32, EPI_STD, 3, H3S_64>(b, st);
    else if (strip && (3 * (a.seg[0].C >> 5)) % b.ksplit == 0)
      rc = launch_conv_h3s_cfg<128, 128, 32, EPI_STD, 3, H3S_128W>(b, st);
    else if (!strip && tile_rows(a) >= 50000)  // big-M stride-2 / two-segment: A from registers
      // (3 blocks / CU, late round 5: 150-153 VGPRs, 722 tiles in one round; per launch within 1 %, bench
      // +0.9 % with two steps in flight, bit-identical: profiles/r05bp_*)
      rc = launch_conv_r3_cfg<128, 128, 32, EPI_STD, 3, 2, R3_BODY>(b, st);
    if (!ok(rc)) {
      b.tile_cnt = nullptr;  // conv_h3: the reduce launch (conv_h3_kernel.h splitk_ticket)
      if ((a.Kpad / 32) % b.ksplit != 0) b.ksplit = 1;  // K not divisible into the slices: no split
      // the FPN low-resolution 1x1 convs left on conv_h3 (level 1's at mask 61): 64 x 128 tiles, 2 x 2 waves,
      // 3 blocks / CU, same K order (late round 5: 23.4 -> 18.0 us, bit-identical, profiles/r05bo_*; the
      // layer3 / 4 convs on the same tiles were slower, r05bn_*)
      if (sliced && a.seg[0].KH == 1 && a.seg[0].KW == 1)
        rc = launch_conv_h3_cfg<64, 128, 32, EPI_STD, 3, 32, 2, false, 2, 1, 64>(b, st);
      if (!ok(rc)) rc = launch_conv_h3_cfg<128, 128, 32, EPI_STD, 2, 32, 2, false, 2, 1>(b, st);
    }
    if (!ok(rc) && !sliced) rc = launch_conv_x6g_cfg<128, 128, 32, EPI_STD, 2, 16, 3, 0, 128, 1>(b, st);
  }
  return rc;
}

int launch_conv(const ConvArgs& a, int epilogue, int math, hipStream_t st) {
  // Host-side shape checks: the kernels assume these and never bounds-check them.
  if (a.N <= 0 || a.N % 64 != 0 || a.M <= 0 || a.Kpad <= 0 || a.Kpad % 16 != 0) {
    set_error("conv: unsupported shape M=%d N=%d Kpad=%d", a.M, a.N, a.Kpad);
    return SFA_E_UNSUPPORTED;
  }
  for (int s = 0; s < a.nseg; ++s) {
    const ConvSeg& g = a.seg[s];
    if (!g.x || g.C < 4 || (g.C & (g.C - 1)) || (1 << g.logC) != g.C || g.KW <= 0 || g.KH <= 0) {
      set_error("conv: bad segment %d (C=%d)", s, g.C);
      return SFA_E_UNSUPPORTED;
    }
    if (g.bytes == 0 || g.bytes >= (1u << 31)) {
      set_error("conv: segment %d input is empty or >= 2 GiB (32-bit buffer offsets)", s);
      return SFA_E_UNSUPPORTED;
    }
    if (g.C < 16 && s != a.nseg - 1) {
      set_error("conv: narrow-channel segment must be last");
      return SFA_E_UNSUPPORTED;
    }
  }
  if (a.nseg == 2 && (a.kseg1 % 16 != 0 || a.kseg1 <= 0 || a.kseg1 >= a.Kpad)) {
    set_error("conv: bad kseg1 %d", a.kseg1);
    return SFA_E_UNSUPPORTED;
  }
  if (a.wstride || a.wk0 || a.res_up) {  // K-sliced weights / half-res residual: conv_h3_kernel only
    if (math != SFA_MATH_FP16X3 || epilogue != EPI_STD) {
      set_error("conv: K-sliced weights / upsampled residual need fp16x3 and the standard epilogue");
      return SFA_E_UNSUPPORTED;
    }
    if (a.res_up && (a.OH % 2 || a.OW % 2 || a.res)) {
      set_error("conv: upsampled residual needs even output dims and no full-res residual");
      return SFA_E_UNSUPPORTED;
    }
    return launch_conv_h3(a, epilogue, st);
  }
  if (math == SFA_MATH_FP16X3) {
    const int rc = launch_conv_h3(a, epilogue, st);
    if (rc != SFA_E_UNSUPPORTED) return rc;
  }
  if (math == SFA_MATH_BF16X6 || math == SFA_MATH_FP16X3) {
    const int rc = launch_conv_x6(a, epilogue, st);
    if (rc != SFA_E_UNSUPPORTED) return rc;
  }
  // Tile choice per shape, from tools/convbench.hip sweeps on MI355X (round 1):
  // 32x64 / 32x32 wave tiles at 4 waves per SIMD hide the gather latency best;
  // BK = 32 pays only for the long-K, few-block layer4 shapes; the LDS-DMA ring
  // (GLDS) gains 2-8 % on the heads and layer3, nothing elsewhere.
  if (epilogue == EPI_HEAD) {
    if (a.N / 64 > SFA_MAX_HEADS) {
      set_error("conv: too many heads");
      return SFA_E_UNSUPPORTED;
    }
    return launch_conv_cfg<128, 64, 32, 64, 16, EPI_HEAD, 4, true>(a, st);
  }
  if (a.N == 64) return launch_conv_cfg<128, 64, 32, 64, 16, EPI_STD, 4>(a, st);
  if (a.N % 128 == 0) {
    if ((tile_rows(a) + 127) / 128 * (a.N / 128) >= 512)
      return launch_conv_cfg<128, 128, 64, 64, 16, EPI_STD, 3>(a, st);
    if ((tile_rows(a) + 63) / 64 * (a.N / 128) >= 512)
      return launch_conv_cfg<64, 128, 32, 64, 16, EPI_STD, 4, true>(a, st);
    if (a.Kpad % 32 == 0 && (a.nseg == 1 || a.kseg1 % 32 == 0))
      return launch_conv_cfg<64, 64, 32, 32, 32, EPI_STD, 4>(a, st);
  }
  return launch_conv_cfg<64, 64, 32, 32, 16, EPI_STD, 4>(a, st);
}

int launch_stem_patch(const ConvArgs& a, hipStream_t st) { return launch_stem_patch_pool(a, st); }

}  // namespace sfa
