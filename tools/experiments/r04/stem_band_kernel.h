// Stem conv 7x7/s2/p3 (3 -> 64) + BN + ReLU + max-pool 3x3/s2/p1 on full-width row bands, fp16x3
// (fpn_resnet.py:120-123,179-182).  Round 4 attempt at VERDICT r03 item 6 (replace
// stem_patch_pool2_kernel + its stem_pool_merge_kernel launch: no side buffer, no merge pass, no
// atomics). ROUND-4 EXPERIMENT, NOT ADOPTED (tools/convbench4 hook only): bit-identical to the patch
// stem, but 210-212 us (one block chain at a time: every A-fragment pair waited for with
// lgkmcnt(0)) and 202-206 us with two blocks' MFMA chains interleaved, against the patch stem's
// 170-183 us + 12 us merge on the same boxes (profiles/r04a_convbench4_stem_regw_tiles.txt,
// r04f_convbench4_stem_band_paired.txt); bench -1.5 % (profiles/r04d_ab_fpn_gemm_stem.txt). Its
// A fragment feeds one 16-channel column block per read (0.67 ds_read_b128 per MFMA, the patch
// stem's 0.44), which the paired chains do not change.
//
// Work.  A block owns the pooled rows [py0, py1) of one frame (a "segment"; frames x segments
// blocks, about one per CU) and walks band tiles of 4 conv rows at FULL width: tile j is conv rows
// c_j = 2 py0 - 1 + 4 j .. c_j + 3.  Tile j completes pooled row py0 + 2 j (conv rows c_j .. c_j + 2,
// all its own) and py0 + 2 j - 1 (conv rows c_j - 2, c_j - 1 — the previous tile's last two, kept
// per column as their max in registers — and c_j).  Full width makes the pool's horizontal halo
// internal; the walk makes the vertical one a register carry; the only recomputation is conv row
// c_0 = 2 py0 - 1, also the previous segment's last.  Every pooled cell is written once, by one
// block, with a plain store.
//
// Input.  A tile reads input rows 2 c_j - 3 .. 2 c_j + 9 (13 rows, columns -3 .. W + 2).  They live in
// an LDS ring of 13 rows, split into fp16 hi / lo at the tile's scale (one 8-B pixel of 4 channels
// per term, channel 3 = 0; rows padded so the A reads are conflict-free).  Consecutive tiles share 5
// rows: a tile adds 8 new rows, prefetched into registers during the previous tile's MFMAs, so a
// segment reads each input byte from HBM once (the first tile's 5 shared rows aside).
//
// Scale.  2^(13 - e) of the TILE's max |x| over its 13 rows (a power of two, like the round-3
// stem's 16 x 16-tile scale: products, f32 sums and the 1 / s rescale are bit-identical whenever
// the lo terms stay normal fp16; the round-3 and round-4 stems give the same bits on every test
// input).  When the scale changes between tiles the 5 shared rows are re-split (reloaded; rare).
//
// MFMA.  8 waves: wave w takes output channels 16 (w & 3) .. + 15 (one column block; its fp16x3
// weights — 7 k-steps x 2 terms — held in 56 VGPRs for the whole kernel) and the half (w >> 2) of
// the band's 4-column blocks.  An M block is 4 rows x 4 columns: A row m =
// (column m >> 2, row m & 3), so accumulator lane (g, c) holds column g's four rows for channel c —
// the pool's vertical maxima are in-lane, the horizontal ones two ds_bpermutes away.  K order
// (kh; kw 0..7, c 0..3; kw = 7 a zero weight column) and the three products per k-step (lo hi,
// hi lo, hi hi) are the round-3 stem's: the same accumulators bit for bit.
#pragma once

#include "../../../lidar-image_object-detection_-fpn_resnet-yolov8_amd/csrc/stem_patch_kernel.h"

namespace sfa {

namespace stem_band {
constexpr int NT = 512, NW = 8;
constexpr int RING = 13;     // input rows of a 4-conv-row tile
constexpr int NEWR = 8;      // rows a tile adds
constexpr int MAX_W = 608;   // widest input (static LDS)
// dwords per ring row and term: (W + 6) pixels x 2 dwords, padded to 8 (mod 32) so the 4 conv rows
// of an M block (ring rows 2 apart) start on bank offsets 0, 16, 32, 48
__host__ __device__ constexpr int pitch_dw(int W) { return 2 * (W + 6) + ((8 - (2 * (W + 6)) % 32) + 32) % 32; }
constexpr int RING_BYTES = RING * 2 * pitch_dw(MAX_W) * 4;
constexpr int XCH_FLOATS = NW * 2 * 16;  // [wave][pooled row A / B][16 channels]: the band's left halo
constexpr int LDS_BYTES = RING_BYTES + XCH_FLOATS * 4 + 2 * NW * 4;
constexpr int NI8 = (NEWR * (MAX_W / 4) + NT - 1) / NT;  // prefetch items per thread (3)
}  // namespace stem_band

// IN: input layout (conv.h StemInput); NBW: 4-column blocks per wave (OW / 8).
template <int IN, int NBW>
__global__ void __launch_bounds__(512, 1) stem_band_kernel(const ConvArgs a, int segs) {
#pragma clang fp contract(off)
  using namespace stem_band;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  const ConvSeg& gs = a.seg[0];
  const int H = gs.H, W = gs.W, OH = a.OH, PH = a.OH >> 1, PW = a.OW >> 1;
  const int NG = W >> 2;  // 4-pixel column groups of an input row
  const int PD = pitch_dw(W), TERMB = PD * 4, ROWB = 2 * TERMB;
  unsigned char* const ring = smem;
  float* const XCH = reinterpret_cast<float*>(smem + RING_BYTES);
  float* const WMX = XCH + XCH_FLOATS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nh = wave & 3, cq = wave >> 2;

  const int b = blockIdx.x / segs, sk = blockIdx.x - b * segs;
  const int py0 = sk * PH / segs, py1 = (sk + 1) * PH / segs;
  const int P = py1 - py0;
  if (P <= 0) return;  // uniform per block
  const int T = (P & 1) ? (P + 1) / 2 : P / 2 + 1;
  const int cr0 = 2 * py0 - 1;  // conv row of tile 0's first row

  // ---- input items: (ring row r of a tile, column group q) -> 4 pixels x 4 channels ----
  auto load_item = [&](int iy, int q, x6_f32x4 (&v)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = x6_f32x4{0.f, 0.f, 0.f, 0.f};
    if ((unsigned)iy < (unsigned)H) {
      if constexpr (IN == STEM_IN_NHWC4) {
        const x6_f32x4* p = reinterpret_cast<const x6_f32x4*>(gs.x) + ((size_t)b * H + iy) * W + 4 * q;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = p[e];
      } else {
        const size_t hw = (size_t)H * W;
        const int sy = IN == STEM_IN_NCHW3_FLIP ? H - 1 - iy : iy;
        const int sx = IN == STEM_IN_NCHW3_FLIP ? W - 4 - 4 * q : 4 * q;
        const float* p = gs.x + (size_t)b * 3 * hw + (size_t)sy * W + sx;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const x6_f32x4 t = *reinterpret_cast<const x6_f32x4*>(p + c * hw);
          v[c] = IN == STEM_IN_NCHW3_FLIP ? x6_f32x4{t[3], t[2], t[1], t[0]} : t;
        }
      }
    }
  };
  auto item_max = [&](const x6_f32x4 (&v)[4]) {
    float m = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[e][0]), fabsf(v[e][1])), fmaxf(fabsf(v[e][2]), fabsf(v[e][3]))));
    return m;
  };
  // pixel 4 q + e of the row -> ring pixel 4 q + 3 + e (ring pixel i = input column i - 3)
  auto write_item = [&](int slot, int q, const x6_f32x4 (&v)[4], float s) {
    unsigned char* row = ring + slot * ROWB + (4 * q + 3) * 8;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const x6_f32x4 px = IN == STEM_IN_NHWC4 ? v[e] : x6_f32x4{v[0][e], v[1][e], v[2][e], 0.f};
      f16x4_t hi, lo;
      split2h(px, s, hi, lo);
      *reinterpret_cast<f16x4_t*>(row + e * 8) = hi;
      *reinterpret_cast<f16x4_t*>(row + TERMB + e * 8) = lo;
    }
  };
  // two per-wave maxima (ring rows < 8 / >= 8 of the items) -> WMX (read after the next barrier)
  auto publish_max = [&](float m0, float m1) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      m0 = fmaxf(m0, __shfl_xor(m0, o, 64));
      m1 = fmaxf(m1, __shfl_xor(m1, o, 64));
    }
    if (lane == 0) {
      WMX[2 * wave] = m0;
      WMX[2 * wave + 1] = m1;
    }
  };
  auto read_max = [&](float& m0, float& m1) {
    m0 = WMX[0];
    m1 = WMX[1];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      m0 = fmaxf(m0, WMX[2 * w]);
      m1 = fmaxf(m1, WMX[2 * w + 1]);
    }
  };
  // input row of ring row r of tile j
  auto in_row = [&](int j, int r) { return 2 * (cr0 + 4 * j) - 3 + r; };

  // ---- prologue: zero column pads, tile 0's 13 rows ----
  for (int i = tid; i < RING * 2 * 6; i += NT) {  // ring pixels 0..2 and W + 3 .. W + 5 of every row / term
    const int r = i / 12, k = i % 12;
    const int term = k / 6, p = k % 6;
    const int px = p < 3 ? p : W + p;
    *reinterpret_cast<uint2*>(ring + r * ROWB + term * TERMB + px * 8) = make_uint2(0u, 0u);
  }
  float sc, ainv;
  {
    const int n0 = RING * NG;
    float m0 = 0.f, m1 = 0.f;
    for (int it0 = 0; it0 < n0; it0 += 2 * NT) {  // two items in flight per thread
      x6_f32x4 v0[4], v1[4];
      const int i0 = it0 + tid, i1 = it0 + NT + tid;
      const int r0 = i0 / NG, r1 = i1 / NG;
      if (i0 < n0) load_item(in_row(0, r0), i0 - r0 * NG, v0);
      if (i1 < n0) load_item(in_row(0, r1), i1 - r1 * NG, v1);
      if (i0 < n0) (r0 < NEWR ? m0 : m1) = fmaxf(r0 < NEWR ? m0 : m1, item_max(v0));
      if (i1 < n0) (r1 < NEWR ? m0 : m1) = fmaxf(r1 < NEWR ? m0 : m1, item_max(v1));
    }
    publish_max(m0, m1);
    __syncthreads();
    float a0, a1;
    read_max(a0, a1);
    sc = amax_scale_bits(__float_as_uint(fmaxf(a0, a1)), ainv);
    for (int it0 = 0; it0 < n0; it0 += 2 * NT) {  // the same loads again (L2), split at the scale
      x6_f32x4 v0[4], v1[4];
      const int i0 = it0 + tid, i1 = it0 + NT + tid;
      const int r0 = i0 / NG, r1 = i1 / NG;
      if (i0 < n0) load_item(in_row(0, r0), i0 - r0 * NG, v0);
      if (i1 < n0) load_item(in_row(0, r1), i1 - r1 * NG, v1);
      if (i0 < n0) write_item(r0, i0 - r0 * NG, v0, sc);
      if (i1 < n0) write_item(r1, i1 - r1 * NG, v1, sc);
    }
  }
  float m812;  // max |x| of the current tile's ring rows 8..12 (the next tile's rows 0..4)
  {
    float a0;
    read_max(a0, m812);
  }

  // ---- weights: this wave's 16 channels, 7 k-steps x 2 terms, in registers ----
  // lane (c16, g) holds B[k = 8 g .. 8 g + 7][n = c16] of k-step kh: kw 2 g, 2 g + 1 x c 0..3
  const int c16 = lane & 15, g = lane >> 4;
  const int nch = 16 * nh + c16;
  f16x8_t whi[7], wlo[7];
#pragma unroll
  for (int kh = 0; kh < 7; ++kh)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint16_t* wr = a.wh + ((size_t)t * 64 + nch) * a.Kpad + (kh * 7 + 2 * g) * 4;
      const uint2 lo4 = *reinterpret_cast<const uint2*>(wr);
      const uint2 hi4 = 2 * g + 1 < 7 ? *reinterpret_cast<const uint2*>(wr + 4) : make_uint2(0u, 0u);
      const x6_u32x4 u = {lo4.x, lo4.y, hi4.x, hi4.y};
      (t == 0 ? whi : wlo)[kh] = __builtin_bit_cast(f16x8_t, u);
    }
  const float bn = a.bias[nch], wv = a.winv[nch];
  __syncthreads();  // tile 0's ring

  // A operand of this lane: pixel (column lc, row lr) of the 4 x 4 block, k-group g
  const int lr = lane & 3, lc = c16 >> 2;
  const int a_col = (2 * lc + 2 * g) * 8;  // + 64 per block (4 conv columns = 8 ring pixels)
  float carry[NBW];                        // max of the previous tile's last two conv rows, per column
#pragma unroll
  for (int k = 0; k < NBW; ++k) carry[k] = 0.f;
  float tmx = 0.f;  // the output max of this block (frame amax for the next conv)
  x6_f32x4 pf[NI8][4];  // (NCHW3: [3] unused)
  float* const ybase = a.y + (size_t)b * PH * PW * 64 + nch;
  // pooled stores: per-tile VGPR offset + the block's column as the SGPR offset (no per-block
  // 64-bit addresses kept live across the unrolled blocks)
  const __amdgpu_buffer_rsrc_t rsy =
      __builtin_amdgcn_make_buffer_rsrc(a.y + (size_t)b * PH * PW * 64, (short)0, PH * PW * 64 * 4, 0x00020000);

  for (int j = 0; j < T; ++j) {
    const int cj = cr0 + 4 * j;
    const int base = (NEWR * j) % RING;
    const bool more = j + 1 < T;
    // prefetch tile j + 1's new rows (its ring rows 5..12) — they land during this tile's MFMAs
    if (more) {
#pragma unroll
      for (int k = 0; k < NI8; ++k) {
        const int it = tid + k * NT;
        const int r = it / NG;
        if (r < NEWR) load_item(in_row(j + 1, 5 + r), it - r * NG, pf[k]);
      }
    }
    int rowoff[7];
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      int s = base + 2 * lr + kh;
      s -= s >= RING ? RING : 0;
      s -= s >= RING ? RING : 0;
      rowoff[kh] = s * ROWB + a_col;
    }
    const float cs = wv * ainv;
    const int pyA = py0 + 2 * j - 1, pyB = py0 + 2 * j;
    const bool stA = j >= 1 && pyA < py1, stB = pyB < py1;
    bool rv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) rv[r] = (unsigned)(cj + r) < (unsigned)OH;
    float left[2] = {0.f, 0.f};  // [row A / B]: column 4 blk - 1 (lane g = 0's)
    // lane g = 0 stores pooled column 2 blk, lane g = 2 column 2 blk + 1 (+ 256 B)
    const int vo[2] = {(pyA * PW * 64 + nch) * 4 + (g == 2 ? 256 : 0), (pyB * PW * 64 + nch) * 4 + (g == 2 ? 256 : 0)};
    float pend[2];               // first block's column-0 partials (cq > 0)

    // epilogue of block k: lane (g, c16) = conv column 4 blk + g, rows cj .. cj + 3, channel 16 nh + c16
    auto epi = [&](const int k, const f32x4_t acc) {
      const int blk = cq * NBW + k;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t = fmaf(acc[r], cs, bn);
        v[r] = rv[r] && t > 0.f ? t : 0.f;  // ReLU; rows outside the map pool as 0 (values >= 0)
        tmx = fmaxf(tmx, v[r]);
      }
      const float rowv[2] = {fmaxf(carry[k], v[0]), fmaxf(fmaxf(v[0], v[1]), v[2])};
      carry[k] = fmaxf(v[2], v[3]);
      // keep the carry and the running max evaluated here: left to itself hipcc defers them and
      // keeps every block's values live (spills at 38 blocks per wave)
      asm volatile("" : "+v"(carry[k]), "+v"(tmx));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float val = rowv[h];
        const float up = __shfl(val, lane + 16, 64);  // column 4 blk + g + 1
        const float dn = __shfl(val, lane - 16, 64);  // column 4 blk + g - 1
        const float l3 = __shfl(val, c16 + 48, 64);   // column 4 blk + 3 (the next block's left)
        const float q0 = fmaxf(val, up);               // lane g = 0: pooled column 2 blk (with left)
        const float q1 = fmaxf(fmaxf(dn, val), up);   // lane g = 2: pooled column 2 blk + 1
        const bool st = h ? stB : stA;
        const bool defer = k == 0 && cq > 0;  // the left neighbour's column 4 blk - 1 arrives through XCH
        if (defer) pend[h] = q0;
        if (st && (g == 2 || (g == 0 && !defer)))
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(g == 0 ? fmaxf(left[h], q0) : q1), rsy, vo[h],
                                                blk * 512, 0);
        left[h] = l3;
        if (k == NBW - 1 && cq == 0 && g == 3) XCH[(wave * 2 + h) * 16 + c16] = val;
      }
    };
    // two blocks' MFMA chains interleaved (k-step kh + 1's A fragments of both read during kh's six
    // MFMAs), then their epilogues in column order: the same products per accumulator, the same bits
    static_assert(NBW % 2 == 0, "blocks per wave in pairs");
#pragma unroll
    for (int k = 0; k < NBW; k += 2) {
      const int blk = cq * NBW + k;
      f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      f16x8_t ah[2][2], al[2][2];  // [k-step parity][block of the pair]
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        ah[0][e] = *reinterpret_cast<const f16x8_t*>(ring + rowoff[0] + (blk + e) * 64);
        al[0][e] = *reinterpret_cast<const f16x8_t*>(ring + rowoff[0] + (blk + e) * 64 + TERMB);
      }
#pragma unroll
      for (int kh = 0; kh < 7; ++kh) {
        if (kh + 1 < 7) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const unsigned char* ap = ring + rowoff[kh + 1] + (blk + e) * 64;
            ah[(kh + 1) & 1][e] = *reinterpret_cast<const f16x8_t*>(ap);
            al[(kh + 1) & 1][e] = *reinterpret_cast<const f16x8_t*>(ap + TERMB);
          }
        }
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[kh & 1][0], whi[kh], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[kh & 1][1], whi[kh], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[kh & 1][0], wlo[kh], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[kh & 1][1], wlo[kh], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[kh & 1][0], whi[kh], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[kh & 1][1], whi[kh], acc1, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      epi(k, acc0);
      __builtin_amdgcn_sched_barrier(0);
      epi(k + 1, acc1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // the next tile's new rows: maxima (ring rows 5..7 | 8..12 of tile j + 1)
    if (more) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      float m0 = 0.f, m1 = 0.f;
#pragma unroll
      for (int k = 0; k < NI8; ++k) {
        const int it = tid + k * NT;
        const int r = it / NG;
        if (r < NEWR) {
          const float m = item_max(pf[k]);
          if (r < 3) m0 = fmaxf(m0, m);
          else m1 = fmaxf(m1, m);
        }
      }
      publish_max(m0, m1);
    }
    __syncthreads();  // B1: tile j's ring reads done, XCH and WMX published
    if (cq > 0) {     // the first block's pooled column 2 blk0 with the left neighbour's column
      const int blk0 = cq * NBW;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if ((h ? stB : stA) && g == 0) {
          const float L = XCH[((wave - 4) * 2 + h) * 16 + c16];
          ybase[((size_t)(h ? pyB : pyA) * PW + 2 * blk0) * 64] = fmaxf(L, pend[h]);
        }
      }
    }
    if (more) {
      float m0, m1;
      read_max(m0, m1);
      float ainv1;
      const float sc1 = amax_scale_bits(__float_as_uint(fmaxf(m812, fmaxf(m0, m1))), ainv1);
      const int base1 = (NEWR * (j + 1)) % RING;
      if (sc1 != sc) {  // re-split the 5 shared rows at the new scale (reloaded; block-uniform)
        const int n5 = 5 * NG;
        for (int it = tid; it < n5; it += NT) {
          const int r = it / NG;
          x6_f32x4 v[4];
          load_item(in_row(j + 1, r), it - r * NG, v);
          int s = base1 + r;
          s -= s >= RING ? RING : 0;
          write_item(s, it - r * NG, v, sc1);
        }
      }
#pragma unroll
      for (int k = 0; k < NI8; ++k) {
        const int it = tid + k * NT;
        const int r = it / NG;
        if (r < NEWR) {
          int s = base1 + 5 + r;
          s -= s >= RING ? RING : 0;
          s -= s >= RING ? RING : 0;
          write_item(s, it - r * NG, pf[k], sc1);
        }
      }
      sc = sc1;
      ainv = ainv1;
      m812 = m1;
      __syncthreads();  // B2: tile j + 1's ring
    }
  }
  if (a.amax_out) {  // the pooled output's max (= the conv's, a pool of values >= 0) for this frame
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) tmx = fmaxf(tmx, __shfl_xor(tmx, o, 64));
    if (lane == 0) WMX[wave] = tmx;
    __syncthreads();
    if (tid == 0) {
      float m = WMX[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) m = fmaxf(m, WMX[w]);
      if (m > 0.f) amax_atomic(a.amax_out, b, m);
    }
  }
}

// Grid = frames x segments (segments = pooled rows split evenly, about one block per CU). Needs the
// fp16x3 split stem weights (Kpad >= 196), conv output width a multiple of 16 with OW / 8 blocks per
// wave in {6, 12, 38} (the instantiated widths: 96, 192, 608 input columns), W <= 608, and 16-B
// aligned input; returns SFA_E_UNSUPPORTED otherwise (the caller then takes the round-3 stem).
inline int launch_stem_band(const ConvArgs& a, hipStream_t st) {
  const ConvSeg& g = a.seg[0];
  const int nbw = a.OW / 8;
  const bool al16 = (reinterpret_cast<uintptr_t>(g.x) & 15) == 0;
  if (!a.wh || !a.winv || a.nseg != 1 || a.N != 64 || g.C != 4 || g.KH != 7 || g.KW != 7 || g.stride != 2 ||
      g.pad != 3 || a.Kpad < 196 || a.OW % 16 != 0 || a.OH % 2 != 0 || a.OH * 2 != g.H || a.OW * 2 != g.W ||
      g.W > stem_band::MAX_W || a.res || !a.relu || !al16 || (nbw != 6 && nbw != 12 && nbw != 38))
    return SFA_E_UNSUPPORTED;
  const int frames = a.M / (a.OH * a.OW);
  const int PH = a.OH / 2;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  if (frames <= 0) return SFA_OK;
  int segs = (ncu + frames - 1) / frames;
  segs = segs < 1 ? 1 : (segs > PH ? PH : segs);
  const dim3 gd((unsigned)(frames * segs)), bd(stem_band::NT);
#define SFA_STEM_BAND(IN_, NBW_) hipLaunchKernelGGL((stem_band_kernel<IN_, NBW_>), gd, bd, 0, st, a, segs)
#define SFA_STEM_BAND_W(IN_)       \
  do {                             \
    if (nbw == 38)                 \
      SFA_STEM_BAND(IN_, 38);      \
    else if (nbw == 12)            \
      SFA_STEM_BAND(IN_, 12);      \
    else                           \
      SFA_STEM_BAND(IN_, 6);       \
  } while (0)
  switch (a.stem_in) {
    case STEM_IN_NCHW3: SFA_STEM_BAND_W(STEM_IN_NCHW3); break;
    case STEM_IN_NCHW3_FLIP: SFA_STEM_BAND_W(STEM_IN_NCHW3_FLIP); break;
    default: SFA_STEM_BAND_W(STEM_IN_NHWC4); break;
  }
#undef SFA_STEM_BAND_W
#undef SFA_STEM_BAND
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

}  // namespace sfa
