// Convolution dispatch: picks the kernel (f32 MFMA or bf16x6) and its tile
// configuration per layer shape (conv_kernel.h, conv_x6_kernel.h).
#include <cstdlib>

#include "conv_kernel.h"
#include "conv_x6_kernel.h"
#include "conv_h3_kernel.h"
#include "conv_h3s_kernel.h"
#include "conv_r3_kernel.h"
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

static int num_cus() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0, n = 0;
    ncu = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
              ? n
              : 256;
  }
  return ncu;
}

// Split-K slices of a 128 x 128-tiled body conv (fp16x3, standard epilogue with bias).
// Default (round 2's rule): 2 slices for the 512-wide convs, combined by splitk_reduce_kernel.
// OPT_CONV_TUNE bit 1024 (experimental, measured slower: model.hip tuned()) combines the slices
// in the kernel (a.tile_cnt: the last slice adds the others' partials) and balances the grid —
// 2 blocks per CU run at once and a block's time is set by its K steps, so the count minimises
// ceil(tiles * ks / slots) / ks (+ 5 % of a block per extra slice) over the divisors of the
// conv's K steps; bits 12..15 force a count. Tiles are priced at 16 frames of the conv's
// geometry, so a frame's arithmetic never depends on its batch.
static int pick_ksplit(const ConvArgs& a, int ksteps, bool inkernel) {
  if (!a.part || !a.bias || a.wstride || a.wk0 || a.res_up) return 1;
  const int forced = (a.tune >> 12) & 15;
  if (forced) return ksteps % forced == 0 ? forced : 1;
  if (!(a.tune & 1024) || !inkernel || !a.tile_cnt) return a.N >= 512 ? 2 : 1;
  const long long tiles = (tile_rows(a) + 127) / 128 * (a.N / 128);
  const long long slots = 2LL * num_cus();
  int best = 1;
  double best_cost = 1e30;
  for (int ks = 1; ks <= 8; ++ks) {
    if (ksteps % ks) continue;
    const double rounds = (double)((tiles * ks + slots - 1) / slots);
    const double cost = rounds / ks + 0.05 * (ks - 1);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = ks;
    }
  }
  return best;
}

// One-segment 3x3 / stride 1 / pad 1 conv with 32-channel chunks: conv_h3s_kernel applies.
static bool strip_ok(const ConvArgs& a) {
  const ConvSeg& g = a.seg[0];
  return a.nseg == 1 && g.KH == 3 && g.KW == 3 && g.stride == 1 && g.pad == 1 && g.C >= 32 &&
         (g.C & 31) == 0 && a.Kpad == 9 * g.C && a.OH == g.H && a.OW == g.W;
}

// fp16x3 tiles per shape (tools/convbench.hip sweeps: profiles/r01_convbench_h3n*.txt,
// r01_convbench_h3m.txt, r01_convbench_strip_splitk.txt):
//  * heads: conv_h3_kernel on 16x16x32 MFMAs, 256x320 (all 5 heads of a level per tile);
//  * 3x3/s1 body convs: conv_h3s_kernel (A staged once per kh as a row strip for the three kw
//    taps): -4..5 % vs per-tap staging; 64-wide: 128x64 at 3 blocks/CU, 128..512-wide: 128x128.
//    In isolation 64x128 tiles with 16-row wave tiles at 3 blocks/CU are 7-8 % faster on
//    layer2/3 (profiles/r01_convbench_strip_tiles.txt) and the single-flight forward gains
//    ~60 us, but with two steps in flight the bench loses ~1 % (profiles/r01_ab_strip_tiles.txt):
//    kept selectable (SFA_TUNE bit 2), not the default;
//  * the rest (stride-2 convs, 2-segment convs, 1x1 FPN convs, the stem): conv_h3_kernel,
//    16x16x32 for the 64-wide ones, 32x32x16 for the 128..512-wide ones, BK 16 for the stem;
//  * round 2: conv_r3_kernel (conv_r3_kernel.h: A fragments loaded straight into registers,
//    only W through LDS, W DMA spread over the column blocks, transposed accumulators) for the
//    heads and the big-M (layer2) convs the strip kernel cannot take (stride 2, conv +
//    downsample segments); on layer3/4 shapes it does not beat the strip / conv_h3 kernels. The
//    strip kernel runs in the transposed-accumulator form too (float4 epilogue: -7..11 %;
//    profiles/r02_convbench_*.txt). SFA_TUNE bits 4 / 8 / 16 return the heads / the big-M
//    non-strip convs / the strip convs to the round-1 kernels for same-box A/B, bit 32 the FPN
//    skip convs, bit 64 the heads to the unpacked epilogue, bit 128 the 64-wide strip convs to
//    no residual prefetch, bit 256 the conv_r3 launches to the tap-major K order, bit 512 the
//    128..512-wide conv_h3 launches to the 32x32x16 MFMA form; round 3: bit 65536 the heads to
//    the unstaggered kernel, bit 131072 to the stagger without s_setprio;
//  * split-K 2 for the 512-wide (layer4) convs, whose 184 tiles cannot fill 256 CUs (-13..16 %);
//    picked from the width only, so a frame's arithmetic never depends on the batch.
// conv_x6g_kernel<..., PREC 1> tiles as the fallback.
// Tuning knob for same-box A/B runs and the kernel-equivalence tests: ConvArgs::tune, set from
// the model handle (sfa_model_set_option(SFA_OPT_CONV_TUNE); env SFA_TUNE seeds it when the
// model is created), 0 = the defaults below. A captured graph keeps the kernels chosen at
// capture time.

// conv_r3_kernel variants (conv_r3_kernel.h ABL bits): W DMA spread over the column blocks (256),
// transposed accumulators with float4 / permlane-swap epilogues (2048); heads also s_setprio 1
// for the second half of the waves (4).
// 524288: channel-chunk-major K order (the 3x3 window's 32-channel slices stay in L2 across the 9
// taps; heads' HBM traffic 3.5-4.7x lower, -3..7 % per launch: profiles/r02_convbench_cmaj.txt)
constexpr int R3_BODY = 256 | 2048 | 524288;
constexpr int R3_FPN = 256 | 2048 | 32768;  // + the upsampled-residual epilogue (FPN skip convs)
// strip kernel (conv_h3s_kernel.h ABL bits): transposed epilogue (2), v_fma_mix split (8); the
// 64-wide also pre-split strip (4) and the residual tile loaded during the last super-step (128).
// Non-temporal output stores (strip 2048, r3 262144) are 1-6 % faster per launch in isolation but
// 1.2 % slower end to end (the next conv then reads its input from HBM): not used.
constexpr int H3S_64 = 2 | 4 | 8 | 128;
constexpr int H3S_128 = 2 | 8;
constexpr int R3_HEAD = 256 | 2048 | 4 | 4096 | 8192 | 16384 | 65536 | 524288;  // + v_fma_mix split, 3-block W
                                                                                 // read-ahead, scalar tap decode,
                                                                                 // packed epilogue, chunk-major K
// + waves 4-7 half a K-tile behind their SIMD partners (three W stages): heads L1 / L2 / L0
// -4.6 / -3.1 / -1.0 % per launch in isolation, bit-identical (profiles/r03h_convbench_heads_stagger.txt)
constexpr int R3_HEAD_STAG = R3_HEAD | 1048576;

static int launch_conv_h3(const ConvArgs& a, int epilogue, hipStream_t st) {
  if (!a.wh || !a.winv) return SFA_E_UNSUPPORTED;
  auto ok = [](int rc) { return rc != SFA_E_UNSUPPORTED; };
  int rc = SFA_E_UNSUPPORTED;
  const bool sliced = a.wstride || a.wk0 || a.res_up;  // conv_h3_kernel reads these; the others do not
  const bool strip = strip_ok(a) && !sliced;
  if (epilogue == EPI_HEAD) {
    if (a.N == 320) {
      if (a.tune & 64)  // the unpacked head epilogue (A/B)
        rc = launch_conv_r3_cfg<256, 320, 32, EPI_HEAD, 1, 2, R3_HEAD & ~65536>(a, st);
      else if (a.tune & 256)  // tap-major K order (A/B)
        rc = launch_conv_r3_cfg<256, 320, 32, EPI_HEAD, 1, 2, R3_HEAD & ~524288>(a, st);
      else if (a.tune & 65536)  // round 2: no stagger, two W stages, 3-block read-ahead (A/B)
        rc = launch_conv_r3_cfg<256, 320, 32, EPI_HEAD, 1, 2, R3_HEAD>(a, st);
      else if (a.tune & 131072)  // stagger without the second half's s_setprio (A/B)
        rc = launch_conv_r3_cfg<256, 320, 32, EPI_HEAD, 1, 3, R3_HEAD_STAG & ~4>(a, st);
      else if ((a.tune & 33554432) && tile_rows(a) < 200000)
        // round 3 (A/B): the level-0 heads (76 x 76) on 192 x 320 tiles of twelve 16-row waves, three
        // per SIMD: 482 tiles fill 256 CUs 1.88 times instead of 361 tiles 1.41 times (same per-element
        // K order: the same bits)
        rc = launch_conv_r3_cfg<192, 320, 16, EPI_HEAD, 1, 3, R3_HEAD_STAG>(a, st);
      else if (a.tune & 16777216)  // round 3: shifted A fragments for taps kw 1, 2 (A/B)
        rc = launch_conv_r3_cfg<256, 320, 32, EPI_HEAD, 1, 3, R3_HEAD_STAG | 8388608>(a, st);
      else if (!(a.tune & 4))
        rc = launch_conv_r3_cfg<256, 320, 32, EPI_HEAD, 1, 3, R3_HEAD_STAG>(a, st);
      if (!ok(rc)) rc = launch_conv_h3_cfg<256, 320, 32, EPI_HEAD, 1, 32, 2, false, 2, 1>(a, st);
      if (!ok(rc)) rc = launch_conv_x6g_cfg<256, 320, 32, EPI_HEAD, 1, 16, 3, 0, 320, 1>(a, st);
    }
    if (!ok(rc)) rc = launch_conv_x6g_cfg<256, 64, 32, EPI_HEAD, 1, 16, 3, 0, 64, 1>(a, st);
    return rc;
  }
  if (a.res_up && !(a.tune & 32) && (a.tune & 1048576)) {  // A/B: the residual's taps before the K loop
    if (a.N == 64)
      rc = launch_conv_r3_cfg<128, 64, 32, EPI_STD, 3, 2, R3_FPN | 4194304>(a, st);
    else if (a.N % 128 == 0)
      rc = launch_conv_r3_cfg<128, 128, 32, EPI_STD, 2, 2, R3_FPN | 4194304>(a, st);
    if (ok(rc)) return rc;
  }
  if (a.res_up && !(a.tune & 32)) {  // FPN skip convs: transposed float4 epilogue, float4 taps
    if (a.N == 64)
      rc = launch_conv_r3_cfg<128, 64, 32, EPI_STD, 4, 2, R3_FPN>(a, st);
    else if (a.N % 128 == 0)
      rc = launch_conv_r3_cfg<128, 128, 32, EPI_STD, 2, 2, R3_FPN>(a, st);
    if (ok(rc)) return rc;
  }
  if (a.N == 64) {
    if (strip) {
      if (a.tune & 16) rc = launch_conv_h3s_cfg<128, 64, 32, EPI_STD, 3>(a, st);
      else if (a.tune & 1) rc = launch_conv_h3s_cfg<128, 64, 32, EPI_STD, 3, 2>(a, st);
      else if (a.tune & 128) rc = launch_conv_h3s_cfg<128, 64, 32, EPI_STD, 3, 14>(a, st);  // round-2 A/B
      else rc = launch_conv_h3s_cfg<128, 64, 32, EPI_STD, 3, H3S_64>(a, st);
    }
    if (!ok(rc) && a.Kpad >= 256) rc = launch_conv_h3_cfg<256, 64, 32, EPI_STD, 1, 32, 2, false, 0, 1>(a, st);
    if (!ok(rc)) rc = launch_conv_h3_cfg<128, 64, 32, EPI_STD, 2, 16, 3, false, 0>(a, st);
    if (!ok(rc) && !sliced) rc = launch_conv_x6g_cfg<256, 64, 32, EPI_STD, 1, 16, 3, 0, 64, 1>(a, st);
    return rc;
  }
  if (a.N % 128 == 0) {
    ConvArgs b = a;
    const bool r3_big = !strip && tile_rows(a) >= 50000 && !(a.tune & 8);  // conv_r3 below: in-kernel split
    if (strip)
      b.ksplit = pick_ksplit(a, 3 * (a.seg[0].C >> 5), !(a.tune & 16) && !(a.tune & 2));
    else
      b.ksplit = pick_ksplit(a, a.Kpad / 32, r3_big);
    if (strip) {
      // A/B (round 3): 256 x 128 strip tiles, one 8-wave block per CU (half the W DMA per output
      // row; same per-element summation order, so the same bits) for the 256-wide (bit 2097152)
      // / 128-wide (bit 8388608) unsplit strip convs
      const bool s256 = b.ksplit == 1 && ((a.N == 256 && (a.tune & 2097152)) || (a.N == 128 && (a.tune & 8388608)));
      if (a.tune & 16)
        rc = launch_conv_h3s_cfg<128, 128, 32, EPI_STD, 2>(b, st);
      else if (s256)
        rc = launch_conv_h3s_cfg<256, 128, 32, EPI_STD, 1, H3S_128>(b, st);
      else if (a.tune & 2)
        rc = launch_conv_h3s_cfg<64, 128, 16, EPI_STD, 3, 10>(b, st);
      if (!ok(rc)) rc = launch_conv_h3s_cfg<128, 128, 32, EPI_STD, 2, H3S_128>(b, st);
    } else if (tile_rows(a) >= 50000 && !(a.tune & 8)) {  // big-M stride-2 / two-segment: A from registers
      if (a.tune & 256)  // tap-major K order (A/B)
        rc = launch_conv_r3_cfg<128, 128, 32, EPI_STD, 2, 2, R3_BODY & ~524288>(b, st);
      else
        rc = launch_conv_r3_cfg<128, 128, 32, EPI_STD, 2, 2, R3_BODY>(b, st);
    }
    if (!ok(rc)) {
      // 16x16x32 MFMA form (round 2): -6 % per launch on layer3.0.conv1, +1.2 % end to end
      // (profiles/r02_ab_h3_mf1.txt); SFA_TUNE bit 512 returns to the 32x32x16 form
      if (a.tune & 512)
        rc = launch_conv_h3_cfg<128, 128, 32, EPI_STD, 2, 32, 2, false, 2>(b, st);
      else
        rc = launch_conv_h3_cfg<128, 128, 32, EPI_STD, 2, 32, 2, false, 2, 1>(b, st);
    }
    if (!ok(rc) && b.ksplit > 1) {  // K not divisible into the slices: no split
      b.ksplit = 1;
      if (strip) rc = launch_conv_h3s_cfg<128, 128, 32, EPI_STD, 2>(b, st);
      if (!ok(rc)) rc = launch_conv_h3_cfg<128, 128, 32, EPI_STD, 2, 32, 2, false, 2>(b, st);
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
  if (epilogue == EPI_POOL) {  // fused stem + max-pool: fp16x3 only; the caller falls back
    if (math != SFA_MATH_FP16X3 || !a.wh || !a.winv || a.nseg != 1 || a.N != 64 || !a.relu || a.res ||
        a.ksplit > 1 || a.OH % 8 != 0 || a.OW % 16 != 0) {
      set_error("conv: fused max-pool epilogue unsupported here (OH=%d OW=%d N=%d)", a.OH, a.OW, a.N);
      return SFA_E_UNSUPPORTED;
    }
    return launch_conv_h3_cfg<128, 64, 32, EPI_POOL, 2, 16, 3, false, 0, 0>(a, st);  // the stem's tile
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

// The three KFPN levels' heads in one launch (conv_r3_group_kernel: longest K first, so the
// per-level launches' partial last rounds of tiles become one short tail). fp16x3 and the
// default head kernel only; SFA_E_UNSUPPORTED otherwise (the caller launches per level).
int launch_conv_heads_group(const ConvArgs* lv, int n, int math, hipStream_t st) {
  if (math != SFA_MATH_FP16X3 || n != 3) return SFA_E_UNSUPPORTED;
  for (int i = 0; i < n; ++i) {
    if (!lv[i].wh || !lv[i].winv || lv[i].N != 320 || lv[i].tune != lv[0].tune) return SFA_E_UNSUPPORTED;
  }
  if (lv[0].tune & (4 | 64 | 256 | 65536 | 131072 | 16777216 | 33554432))
    return SFA_E_UNSUPPORTED;  // per-level A/B head kernels
  return launch_conv_r3_group_cfg<256, 320, 32, 1, 3, R3_HEAD_STAG>(lv, n, st);
}

int launch_stem_patch(const ConvArgs& a, hipStream_t st) { return launch_stem_patch_pool(a, st); }

}  // namespace sfa
