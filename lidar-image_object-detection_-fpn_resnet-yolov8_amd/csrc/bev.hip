// BEV voxelisation: get_filtered_lidar + makeBEVMap on the GPU.
//
// Reference: data_process/kitti_data_utils.py:228-251 (filter),
//            data_process/kitti_bev_utils.py:22-55 (makeBEVMap).
//
// Default: the binned path (count / scan / bin / strip kernels below): points binned by 8-row
// strips of the map, each strip's top keys and counts reduced in LDS. For batches whose points
// do not fit the scratch as records, and as SFA_BEV_ATOMIC=1, the global-atomic path:
// two passes, HBM/atomic bound (SURVEY §8(a) row a1'):
//   pass 1 (one thread per point): inclusive f32 box test, z' = z - minZ (f32),
//     cell = (floor(x/D), trunc(floor(y/D) + 304.5)) with IEEE f32 division,
//     atomicMax of a 64-bit key (bits(z') << 32 | ~index) — z' >= +0 so the
//     float bits are monotone; the max key is the max z with ties broken by the
//     FIRST point in input order, exactly the row np.unique(return_index) picks
//     after the stable lexsort((-z, col, row)) — and atomicAdd of the count.
//   pass 2 (one thread per BEV cell): intensity = i[top], height = z'/4.0 (f32),
//     density = min(1, ln(count+1)/ln 64) (f64 table), written in the requested
//     layout; the scratch cell is re-zeroed for the next call.
// The result is independent of atomic arrival order: bit-exact.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "aux_kernels.h"
#include "common.h"

namespace sfa {

constexpr int kBevH = 608;
constexpr int kBevW = 608;
constexpr int kBevCells = kBevH * kBevW;

struct BevArgs {
  int64_t start[SFA_BEV_MAX_BATCH + 1];
  float minX, maxX, minY, maxY, minZ, maxZ;
  float disc;        // f32(50/608)
  float half_w;      // (BEV_W + 1) / 2 = 304.5
  float max_height;  // f32(float(abs(maxZ - minZ)))
  double density[64];  // min(1, ln(c+1)/ln 64), c = 0..63 (c >= 63 -> 1)
};

// The cell and the 64-bit top-point key of point i of a frame (false: the point is dropped).
template <bool RAW>
__device__ __forceinline__ bool bev_point_cell(const float4 p, const BevArgs& a, int64_t i, int& cell,
                                               unsigned long long& key) {
  float zr = p.z;
  if (RAW) {
    // kitti_data_utils.py:237-239 — inclusive on both ends, NaN fails.
    if (!(p.x >= a.minX && p.x <= a.maxX && p.y >= a.minY && p.y <= a.maxY && p.z >= a.minZ &&
          p.z <= a.maxZ))
      return false;
    zr = __fsub_rn(p.z, a.minZ);  // :241
  } else if (!(zr >= 0.f)) {
    // makeBEVMap on already-filtered points: z is >= 0 after the filter; a negative or
    // NaN z has no defined top-point order (the 64-bit key needs z >= +0) -> skipped.
    return false;
  }
  int row = (int)floorf(__fdiv_rn(p.x, a.disc));                      // kitti_bev_utils.py:28
  int col = (int)__fadd_rn(floorf(__fdiv_rn(p.y, a.disc)), a.half_w);  // :29 (np.int_ truncates)
  // numpy fancy indexing wraps negative indices of the (609, 609) maps (:44-48).
  if (row < 0) row += kBevH + 1;
  if (col < 0) col += kBevW + 1;
  // :50-53 crop to [:608, :608]; indices outside the (609, 609) table (IndexError in
  // numpy) cannot occur after the filter and are skipped for pre-filtered input.
  if (row < 0 || row >= kBevH || col < 0 || col >= kBevW) return false;
  cell = row * kBevW + col;
  key = ((unsigned long long)__float_as_uint(zr) << 32) | (unsigned)(~(unsigned)i);
  return true;
}

template <bool RAW>
__global__ void __launch_bounds__(256) bev_scatter_kernel(const float4* __restrict__ pts,
                                                          BevArgs a,
                                                          unsigned long long* __restrict__ keys,
                                                          unsigned* __restrict__ counts) {
  const int b = blockIdx.y;
  const int64_t s = a.start[b];
  const int64_t n = a.start[b + 1] - s;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int cell;
  unsigned long long key;
  if (!bev_point_cell<RAW>(pts[s + i], a, i, cell, key)) return;
  atomicMax(keys + (size_t)b * kBevCells + cell, key);
  atomicAdd(counts + (size_t)b * kBevCells + cell, 1u);
}

// One output cell: intensity = i[top], height = z'/4.0 (f32), density from the count (f64
// table), stored in the requested layout (torch.flip(bev, [1, 2]) when FLIP).
template <int LAYOUT, bool FLIP>
__device__ __forceinline__ void bev_store_cell_i(const BevArgs& a, int b, int cell, unsigned cnt,
                                                 unsigned long long key, float inten, void* __restrict__ out) {
  float height = 0.f;
  double dens = 0.0;
  if (cnt) {
    const float zr = __uint_as_float((unsigned)(key >> 32));
    height = __fdiv_rn(zr, a.max_height);  // :43-44, f32 division
    dens = a.density[cnt < 63u ? cnt : 63u];
  } else {
    inten = 0.f;
  }
  // torch.flip(bev, [1, 2]): cell (r, c) lands at (607 - r, 607 - c)
  const int oc = FLIP ? kBevCells - 1 - cell : cell;
  if (LAYOUT == SFA_BEV_NHWC4_F32) {
    float4 v = make_float4(inten, height, (float)dens, 0.f);
    reinterpret_cast<float4*>(out)[(size_t)b * kBevCells + oc] = v;
  } else if (LAYOUT == SFA_BEV_NCHW3_F32) {
    float* o = reinterpret_cast<float*>(out) + (size_t)b * 3 * kBevCells + oc;
    o[0] = inten;
    o[kBevCells] = height;
    o[2 * kBevCells] = (float)dens;
  } else {
    double* o = reinterpret_cast<double*>(out) + (size_t)b * 3 * kBevCells + oc;
    o[0] = (double)inten;
    o[kBevCells] = (double)height;
    o[2 * kBevCells] = dens;
  }
}

// intensity = i of the cell's top point (the point index is the low word of the key)
__device__ __forceinline__ float bev_top_intensity(const float4* __restrict__ pts, const BevArgs& a, int b,
                                                   unsigned cnt, unsigned long long key) {
  return cnt ? pts[a.start[b] + ~(unsigned)(key & 0xffffffffull)].w : 0.f;
}

template <int LAYOUT, bool FLIP>
__device__ __forceinline__ void bev_store_cell(const float4* __restrict__ pts, const BevArgs& a, int b, int cell,
                                               unsigned cnt, unsigned long long key, void* __restrict__ out) {
  bev_store_cell_i<LAYOUT, FLIP>(a, b, cell, cnt, key, bev_top_intensity(pts, a, b, cnt, key), out);
}

template <int LAYOUT, bool FLIP>
__global__ void __launch_bounds__(256) bev_gather_kernel(const float4* __restrict__ pts, BevArgs a,
                                                         unsigned long long* __restrict__ keys,
                                                         unsigned* __restrict__ counts,
                                                         void* __restrict__ out) {
  const int b = blockIdx.y;
  const int cell = blockIdx.x * blockDim.x + threadIdx.x;
  if (cell >= kBevCells) return;
  const size_t sc = (size_t)b * kBevCells + cell;
  const unsigned cnt = counts[sc];
  unsigned long long key = 0ull;
  if (cnt) {
    key = keys[sc];
    keys[sc] = 0ull;  // leave scratch zeroed for the next call
    counts[sc] = 0u;
  }
  bev_store_cell<LAYOUT, FLIP>(pts, a, b, cell, cnt, key, out);
}

// ------------------------------------------------------------ binned path --
// The default when the batch's points fit the scratch as records (any KITTI-sized sweep).
// The atomic path above does two device-scope atomics per kept point on a 12-B-per-cell
// scratch spread over the whole map: each is an L2 miss on its own line (the scatter was
// 58 us for 16 sweeps, the gather 38 us). Here the points are binned by 8-row strips of
// the map (76 per frame) and each strip is reduced in LDS:
//   count   per point: its strip; LDS histogram per block, one global add per strip
//   scan    strip offsets in (frame, strip) order (one small block)
//   bin     per point again: a slot in its strip's range (LDS-aggregated reservations),
//           record = {key (8 B), cell within the strip, 0}
//   strip   per (frame, strip): ds_max_u64 / ds_add_u32 over its records in LDS (4,864
//           cells: 58 KiB), then every cell of the strip written in the output layout.
// The same keys and counts reach every cell (max and + are order-free): bit-identical to the
// atomic path. Self-cleaning like it: the strip pass zeroes its strip's counters. The records
// have their own region after the atomic path's keys / counts (round 3: they used to overlap
// them, so every record read was written back as zero — 16 B per point of extra traffic).
constexpr int kStripRows = 8;
constexpr int kStripCells = kStripRows * kBevW;   // 4,864
constexpr int kStrips = kBevH / kStripRows;       // 76
constexpr int kStripThreads = 512;

struct BinScratch {
  unsigned* count;   // [B][kStrips] points per strip
  unsigned* offset;  // [B][kStrips] first record of the strip
  unsigned* cursor;  // [B][kStrips] next free record (reservation counter)
  uint4* rec;        // records
};

constexpr int kBinPPT = 4;  // points per thread of the count / bin passes (strided by the block)

template <bool RAW>
__global__ void __launch_bounds__(256) bev_bin_count_kernel(const float4* __restrict__ pts, BevArgs a,
                                                            BinScratch bs) {
  __shared__ unsigned hist[kStrips];
  const int b = blockIdx.y;
  const int64_t s = a.start[b];
  const int64_t n = a.start[b + 1] - s;
  for (int t = threadIdx.x; t < kStrips; t += blockDim.x) hist[t] = 0u;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kBinPPT; ++j) {
    const int64_t i = ((int64_t)blockIdx.x * kBinPPT + j) * blockDim.x + threadIdx.x;
    int cell;
    unsigned long long key;
    if (i < n && bev_point_cell<RAW>(pts[s + i], a, i, cell, key)) atomicAdd(&hist[cell / kStripCells], 1u);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < kStrips; t += blockDim.x)
    if (hist[t]) atomicAdd(&bs.count[b * kStrips + t], hist[t]);
}

// one block: the exclusive scan of the (frame, strip) counts in that order -> record offsets
// (thread t owns up to kScanPer consecutive bins; wave-level then block-level scan)
constexpr int kScanThreads = 1024;
constexpr int kScanPer = (SFA_BEV_MAX_BATCH * kStrips + kScanThreads - 1) / kScanThreads;
__global__ void __launch_bounds__(kScanThreads) bev_bin_scan_kernel(BinScratch bs, int batch) {
  __shared__ unsigned wsum[kScanThreads / 64];
  const int nbin = batch * kStrips, t = threadIdx.x, lane = t & 63, w = t >> 6;
  unsigned v[kScanPer], sum = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    const int i = t * kScanPer + j;
    v[j] = i < nbin ? bs.count[i] : 0u;
    sum += v[j];
  }
  unsigned inc = sum;  // inclusive scan of the thread sums within the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned o = __shfl_up(inc, d, 64);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  if (w == 0) {
    unsigned x = lane < kScanThreads / 64 ? wsum[lane] : 0u, xi = x;
#pragma unroll
    for (int d = 1; d < kScanThreads / 64; d <<= 1) {
      const unsigned o = __shfl_up(xi, d, 64);
      if (lane >= d) xi += o;
    }
    if (lane < kScanThreads / 64) wsum[lane] = xi - x;  // exclusive wave offsets
  }
  __syncthreads();
  unsigned run = wsum[w] + inc - sum;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    const int i = t * kScanPer + j;
    if (i < nbin) {
      bs.offset[i] = run;
      bs.cursor[i] = run;
    }
    run += v[j];
  }
}

template <bool RAW>
__global__ void __launch_bounds__(256) bev_bin_kernel(const float4* __restrict__ pts, BevArgs a, BinScratch bs) {
  __shared__ unsigned hist[kStrips], base[kStrips];
  const int b = blockIdx.y;
  const int64_t s = a.start[b];
  const int64_t n = a.start[b + 1] - s;
  for (int t = threadIdx.x; t < kStrips; t += blockDim.x) hist[t] = 0u;
  __syncthreads();
  int cell[kBinPPT], strip[kBinPPT];
  unsigned long long key[kBinPPT];
  unsigned slot[kBinPPT];
  bool ok[kBinPPT];
#pragma unroll
  for (int j = 0; j < kBinPPT; ++j) {
    const int64_t i = ((int64_t)blockIdx.x * kBinPPT + j) * blockDim.x + threadIdx.x;
    ok[j] = i < n && bev_point_cell<RAW>(pts[s + i], a, i, cell[j], key[j]);
    strip[j] = ok[j] ? cell[j] / kStripCells : 0;
    slot[j] = ok[j] ? atomicAdd(&hist[strip[j]], 1u) : 0u;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < kStrips; t += blockDim.x)
    base[t] = hist[t] ? atomicAdd(&bs.cursor[b * kStrips + t], hist[t]) : 0u;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kBinPPT; ++j)
    if (ok[j])
      bs.rec[base[strip[j]] + slot[j]] = make_uint4((unsigned)(key[j] & 0xffffffffull), (unsigned)(key[j] >> 32),
                                                    (unsigned)(cell[j] - strip[j] * kStripCells), 0u);
}

template <int LAYOUT, bool FLIP>
__global__ void __launch_bounds__(kStripThreads) bev_strip_kernel(const float4* __restrict__ pts, BevArgs a,
                                                                  BinScratch bs, void* __restrict__ out) {
  __shared__ unsigned long long skey[kStripCells];
  __shared__ unsigned scnt[kStripCells];
  const int strip = blockIdx.x, b = blockIdx.y, bin = b * kStrips + strip;
  for (int c = threadIdx.x; c < kStripCells; c += kStripThreads) {
    skey[c] = 0ull;
    scnt[c] = 0u;
  }
  __syncthreads();
  const unsigned off = bs.offset[bin], cnt = bs.count[bin];
  for (unsigned r = threadIdx.x; r < cnt; r += kStripThreads) {
    const uint4 rec = bs.rec[off + r];
    atomicMax(&skey[rec.z], ((unsigned long long)rec.y << 32) | rec.x);
    atomicAdd(&scnt[rec.z], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    bs.count[bin] = 0u;
    bs.offset[bin] = 0u;
    bs.cursor[bin] = 0u;
  }
  for (int c = threadIdx.x; c < kStripCells; c += kStripThreads)
    bev_store_cell<LAYOUT, FLIP>(pts, a, b, strip * kStripCells + c, scnt[c], skey[c], out);
}

// ------------------------------------------------------- blocked-bin path --
// Round 3 default: ONE pass over the points. Bin-pass block j of a frame takes its points
// [1024 j, 1024 j + 1024) and writes their records into ITS OWN 1024-record region, grouped by
// strip (LDS histogram, exclusive scan, LDS slot per point), plus one word per strip into a
// table: (first record of the strip in the region) | (count << 16). The strip pass for
// (frame, strip) reads the frame's table column and reduces those runs in LDS. No count pass,
// no global scan, no global reservation atomics, and nothing to re-zero: the region and the
// table are written before they are read. Region j of frame b starts at record
// 1024 * (blk0[b] + j), blk0 = the exclusive sum of the frames' ceil(n / 1024) (host).
// Strips of SR map rows: SR = 4 (default, round 3c) — 2,432-cell strips, 35 KiB of LDS per
// 256-thread strip block, four blocks per CU — or SR = 8 (round 3a, SFA_BEV_STRIP8: 71 KiB,
// two 512-thread blocks per CU). The table is stored strip-major (tab[strip][global region]),
// so a strip block reads its column as one contiguous run, once. A record is 8 B: the top-point
// key's z bits and (point index within its 1024-point region << 13 | cell within the strip) —
// the region is the one the strip block found the record in, so the 64-bit key (z bits << 32 |
// ~frame index) is rebuilt exactly (round 3a's 16-B records also carried the cell and the
// intensity, which the strip pass takes from the top point).
constexpr int kBlkPts = 1024;
constexpr int kBlkThreads = 256;
constexpr int kBlkPPT = kBlkPts / kBlkThreads;  // 4

template <int SR>
struct BlkGeom {
  static constexpr int strips = kBevH / SR;         // 152 / 76
  static constexpr int cells = SR * kBevW;          // 2,432 / 4,864
  static constexpr int threads = SR == 8 ? 512 : 256;
  static constexpr int max_regions = SR == 8 ? 2048 : 1024;  // regions of one frame a strip block indexes
};

constexpr int kBlkCellBits = 13;  // cell within a strip (< 4,864)
static_assert(BlkGeom<8>::cells <= (1 << kBlkCellBits) && kBlkPts <= (1 << (32 - kBlkCellBits)), "record packing");

struct BlkScratch {
  uint2* rec;         // [total blocks][kBlkPts]: z bits, (index in region << 13) | cell in strip
  unsigned* tab;      // [strips][total blocks]: first | count << 16
  int nblk_total;     // total blocks (regions) of the batch: the table's row length
  int blk0[SFA_BEV_MAX_BATCH + 1];
};

template <bool RAW, int SR>
__global__ void __launch_bounds__(kBlkThreads) bev_blk_bin_kernel(const float4* __restrict__ pts, BevArgs a,
                                                                  BlkScratch bs) {
  constexpr int NS = BlkGeom<SR>::strips, SC = BlkGeom<SR>::cells;
  constexpr int P = (NS + 63) / 64;  // strips per lane of the scan
  __shared__ unsigned hist[NS], first[NS];
  const int b = blockIdx.y, j = blockIdx.x;
  const int64_t s = a.start[b];
  const int64_t n = a.start[b + 1] - s;
  if ((int64_t)j * kBlkPts >= n) return;  // past this frame's points (the grid fits the largest)
  for (int t = threadIdx.x; t < NS; t += kBlkThreads) hist[t] = 0u;
  __syncthreads();
  int cell[kBlkPPT], strip[kBlkPPT];
  unsigned long long key[kBlkPPT];
  unsigned slot[kBlkPPT];
  bool ok[kBlkPPT];
#pragma unroll
  for (int q = 0; q < kBlkPPT; ++q) {
    const int64_t i = (int64_t)j * kBlkPts + q * kBlkThreads + threadIdx.x;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < n) p = pts[s + i];
    ok[q] = i < n && bev_point_cell<RAW>(p, a, i, cell[q], key[q]);
    strip[q] = ok[q] ? cell[q] / SC : 0;
    slot[q] = ok[q] ? atomicAdd(&hist[strip[q]], 1u) : 0u;
  }
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan of the strip counts (lane l: strips P l .. P l + P - 1)
    const int l = threadIdx.x;
    unsigned c[P], sum = 0u;
#pragma unroll
    for (int q = 0; q < P; ++q) {
      c[q] = P * l + q < NS ? hist[P * l + q] : 0u;
      sum += c[q];
    }
    unsigned x = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned y = __shfl_up(x, d, 64);
      if (l >= d) x += y;
    }
    unsigned e = x - sum;
#pragma unroll
    for (int q = 0; q < P; ++q) {
      if (P * l + q < NS) first[P * l + q] = e;
      e += c[q];
    }
  }
  __syncthreads();
  const size_t region = (size_t)(bs.blk0[b] + j);
  for (int t = threadIdx.x; t < NS; t += kBlkThreads)
    bs.tab[(size_t)t * bs.nblk_total + region] = first[t] | (hist[t] << 16);
  uint2* rec = bs.rec + region * kBlkPts;
#pragma unroll
  for (int q = 0; q < kBlkPPT; ++q)
    if (ok[q])
      rec[first[strip[q]] + slot[q]] =
          make_uint2((unsigned)(key[q] >> 32),
                     ((unsigned)(q * kBlkThreads + threadIdx.x) << kBlkCellBits) | (unsigned)(cell[q] - strip[q] * SC));
}

// One block per (frame, strip): the strip's records — runs in the bin pass's regions, located by
// a scan of the strip's table column (read once, contiguous) and a binary search over it —
// reduced in LDS (max key and count per cell), then every cell of the strip written, the top
// points' intensities gathered first so all those loads are in flight together. (Measured and
// not adopted: the intensity taken from the records in a second pass over them, no random reads
// of the points — 144 vs 170 MB per call, but 1,024-thread blocks with 90 KiB of LDS, 56 vs 46
// us: profiles/r03f_pmc_bev_blocked_v3_intensity_in_records.json.)
template <int LAYOUT, bool FLIP, int SR>
__global__ void __launch_bounds__(BlkGeom<SR>::threads) bev_blk_strip_kernel(const float4* __restrict__ pts, BevArgs a,
                                                                             BlkScratch bs, void* __restrict__ out) {
  constexpr int NT = BlkGeom<SR>::threads, SC = BlkGeom<SR>::cells, MAXR = BlkGeom<SR>::max_regions;
  constexpr int RPT = MAXR / NT;  // table words per thread (at most)
  __shared__ unsigned long long skey[SC];
  __shared__ unsigned scnt[SC];
  __shared__ unsigned pre[MAXR + 1];  // this strip's records before region r
  __shared__ unsigned short first[MAXR];
  __shared__ unsigned wsum[NT / 64];
  const int strip = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  for (int c = tid; c < SC; c += NT) {
    skey[c] = 0ull;
    scnt[c] = 0u;
  }
  const int nblk = bs.blk0[b + 1] - bs.blk0[b];  // <= MAXR (checked at launch)
  const size_t reg0 = (size_t)bs.blk0[b];
  const unsigned* col = bs.tab + (size_t)strip * bs.nblk_total + reg0;
  // exclusive scan of the regions' counts of this strip: thread t owns regions [t*per, t*per+per)
  const int per = (nblk + NT - 1) / NT;
  unsigned wv[RPT];
  unsigned loc = 0;
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int r = tid * per + q;
    wv[q] = q < per && r < nblk ? col[r] : 0u;
    loc += wv[q] >> 16;
  }
  unsigned x = loc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned y = __shfl_up(x, d, 64);
    if ((tid & 63) >= d) x += y;
  }
  if ((tid & 63) == 63) wsum[tid >> 6] = x;
  __syncthreads();  // also: skey / scnt written
  unsigned run = x - loc;
  for (int w = 0; w < (tid >> 6); ++w) run += wsum[w];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int r = tid * per + q;
    if (q < per && r < nblk) {
      pre[r] = run;
      first[r] = (unsigned short)(wv[q] & 0xffffu);
      run += wv[q] >> 16;
    }
  }
  if (tid == NT - 1) {  // the total: every thread's count
    unsigned t = 0;
    for (int w = 0; w < NT / 64; ++w) t += wsum[w];
    pre[nblk] = t;
  }
  __syncthreads();
  const unsigned total = pre[nblk];
  // every record of the strip, 4 per thread per round: region by binary search over pre, the 4
  // loads in flight together, then the LDS max / add
  for (unsigned base = 0; base < total; base += 4 * NT) {
    uint2 e[4];
    int reg[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned idx = base + u * NT + tid;
      int lo = 0, hi = nblk - 1;  // last region with pre[r] <= idx
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= idx) lo = mid; else hi = mid - 1;
      }
      reg[u] = lo;
      e[u] = idx < total ? bs.rec[(reg0 + lo) * kBlkPts + first[lo] + (idx - pre[lo])] : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (base + u * NT + tid < total) {
        const unsigned c = e[u].y & ((1u << kBlkCellBits) - 1u);
        const unsigned i = (unsigned)reg[u] * kBlkPts + (e[u].y >> kBlkCellBits);  // index within the frame
        atomicMax(&skey[c], ((unsigned long long)e[u].x << 32) | (unsigned)~i);
        atomicAdd(&scnt[c], 1u);
      }
  }
  __syncthreads();
  // every cell of the strip: the top points' intensities gathered first (all loads in flight),
  // then the three channels stored
  constexpr int CPT = (SC + NT - 1) / NT;
  float inten[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    const int c = tid + q * NT;
    inten[q] = c < SC ? bev_top_intensity(pts, a, b, scnt[c], skey[c]) : 0.f;
  }
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    const int c = tid + q * NT;
    if (c < SC) bev_store_cell_i<LAYOUT, FLIP>(a, b, strip * SC + c, scnt[c], skey[c], inten[q], out);
  }
}

}  // namespace sfa

using namespace sfa;

// atomic path: keys + counts per cell; binned path: its counters + records (12 B per cell of
// room: ~277 k points per frame) after them
static size_t bev_atomic_bytes(int batch) {
  return align_up((size_t)batch * kBevCells * sizeof(unsigned long long), 256) +
         align_up((size_t)batch * kBevCells * sizeof(unsigned), 256);
}

extern "C" size_t sfa_bev_scratch_size(int batch) {
  if (batch <= 0) return 0;
  return 2 * bev_atomic_bytes(batch);
}

// The scratch layout is fixed by the scratch's CAPACITY (the largest batch it was sized for), never
// by the batch of the call: keys / counts (atomic path, zero between calls) and the binned path's
// counters (zero between calls) sit at the same offsets for every call, and the record regions
// (written before they are read, left dirty) always lie after them.  A layout by the call's batch
// let a small-batch call's records land inside a later larger call's zero areas.
static int bev_capacity_batch(size_t scratch_bytes) {
  int cap = 0;
  while (cap < SFA_BEV_MAX_BATCH && sfa_bev_scratch_size(cap + 1) <= scratch_bytes) ++cap;
  return cap;
}

extern "C" int sfa_bev_voxelize(const float* points, const int64_t* frame_offsets, int batch,
                                const double* boundary, int flags, int out_layout, void* out,
                                void* scratch, size_t scratch_bytes, void* stream) {
  SFA_CHECK_ARG(batch >= 1 && batch <= SFA_BEV_MAX_BATCH, "bev: batch %d out of [1, %d]", batch,
                SFA_BEV_MAX_BATCH);
  SFA_CHECK_ARG(frame_offsets && boundary && out && scratch, "bev: null argument");
  const int cap = bev_capacity_batch(scratch_bytes);
  if (cap < batch) {
    set_error("bev: scratch of %zu bytes holds %d frames, batch is %d (sfa_bev_scratch_size)", scratch_bytes, cap,
              batch);
    return SFA_E_WORKSPACE;
  }
  SFA_CHECK_ARG(out_layout >= 0 && out_layout <= 2, "bev: bad out_layout %d", out_layout);
  SFA_CHECK_ARG((flags & ~(SFA_BEV_PREFILTERED | SFA_BEV_FLIP_HW | SFA_BEV_FORCE_ATOMIC | SFA_BEV_FORCE_BINNED |
                           SFA_BEV_STRIP8)) == 0,
                "bev: bad flags %d", flags);
  const int flags_in = flags;
  const bool flip = (flags & SFA_BEV_FLIP_HW) != 0;
  const bool force_atomic = (flags & SFA_BEV_FORCE_ATOMIC) != 0;  // the atomic path (A/B, the equivalence test)
  flags &= SFA_BEV_PREFILTERED;
  BevArgs a;
  int64_t max_n = 0;
  for (int b = 0; b <= batch; ++b) {
    a.start[b] = frame_offsets[b];
    if (b > 0) {
      const int64_t n = frame_offsets[b] - frame_offsets[b - 1];
      SFA_CHECK_ARG(n >= 0, "bev: frame_offsets not monotone at %d", b);
      SFA_CHECK_ARG(n < (int64_t)0xffffffff, "bev: frame %d has too many points", b - 1);
      if (n > max_n) max_n = n;
    }
  }
  SFA_CHECK_ARG(frame_offsets[0] >= 0, "bev: negative frame offset");
  SFA_CHECK_ARG(max_n == 0 || points, "bev: null points");
  // Python floats -> f32 as numpy does for f32-array ops (NEP 50 / numpy 1.18 agree).
  a.minX = (float)boundary[0];
  a.maxX = (float)boundary[1];
  a.minY = (float)boundary[2];
  a.maxY = (float)boundary[3];
  a.minZ = (float)boundary[4];
  a.maxZ = (float)boundary[5];
  a.disc = (float)(50.0 / 608.0);  // config/kitti_config.py:47
  a.half_w = 304.5f;
  a.max_height = (float)std::fabs(boundary[5] - boundary[4]);
  for (int c = 0; c < 64; ++c) {
    double v = std::log((double)c + 1.0) / std::log(64.0);
    a.density[c] = c == 0 ? 0.0 : (v < 1.0 ? v : 1.0);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  auto* keys = reinterpret_cast<unsigned long long*>(scratch);
  auto* counts = reinterpret_cast<unsigned*>(
      reinterpret_cast<char*>(scratch) +
      align_up((size_t)cap * kBevCells * sizeof(unsigned long long), 256));
  const float4* p4 = reinterpret_cast<const float4*>(points);
  // blocked-bin path (default) when the batch's regions and table fit the binned scratch
  {
    const bool s8 = (flags_in & SFA_BEV_STRIP8) != 0;
    const int nstrips = s8 ? BlkGeom<8>::strips : BlkGeom<4>::strips;
    const int maxr = s8 ? BlkGeom<8>::max_regions : BlkGeom<4>::max_regions;
    BlkScratch bk;
    int64_t nblk_total = 0;
    for (int b = 0; b < batch; ++b) {
      bk.blk0[b] = (int)nblk_total;
      nblk_total += (frame_offsets[b + 1] - frame_offsets[b] + kBlkPts - 1) / kBlkPts;
    }
    bk.blk0[batch] = (int)nblk_total;
    bk.nblk_total = (int)nblk_total;
    const size_t rec_bytes = align_up((size_t)nblk_total * kBlkPts * sizeof(uint2), 256);
    const size_t tab_bytes = (size_t)nblk_total * nstrips * sizeof(unsigned);
    // after the binned path's (zero) counters, which it must not touch
    const size_t cnt_bytes = 3 * align_up((size_t)cap * kStrips * sizeof(unsigned), 256);
    int max_regions = 0;
    for (int b = 0; b < batch; ++b) max_regions = std::max(max_regions, bk.blk0[b + 1] - bk.blk0[b]);
    if (!force_atomic && !(flags_in & SFA_BEV_FORCE_BINNED) && max_regions <= maxr &&
        cnt_bytes + rec_bytes + tab_bytes <= bev_atomic_bytes(cap)) {
      char* sb = reinterpret_cast<char*>(scratch) + bev_atomic_bytes(cap) + cnt_bytes;
      bk.rec = reinterpret_cast<uint2*>(sb);
      bk.tab = reinterpret_cast<unsigned*>(sb + rec_bytes);
      if (max_n > 0) {
        dim3 g1((unsigned)((max_n + kBlkPts - 1) / kBlkPts), batch);
        if (flags == SFA_BEV_RAW) {
          if (s8) hipLaunchKernelGGL((bev_blk_bin_kernel<true, 8>), g1, dim3(kBlkThreads), 0, st, p4, a, bk);
          else hipLaunchKernelGGL((bev_blk_bin_kernel<true, 4>), g1, dim3(kBlkThreads), 0, st, p4, a, bk);
        } else {
          if (s8) hipLaunchKernelGGL((bev_blk_bin_kernel<false, 8>), g1, dim3(kBlkThreads), 0, st, p4, a, bk);
          else hipLaunchKernelGGL((bev_blk_bin_kernel<false, 4>), g1, dim3(kBlkThreads), 0, st, p4, a, bk);
        }
        SFA_LAUNCH_CHECK();
      }
      dim3 g3(nstrips, batch);
#define SFA_BEV_BLK(L, F)                                                                                    \
  do {                                                                                                      \
    if (s8)                                                                                                 \
      hipLaunchKernelGGL((bev_blk_strip_kernel<L, F, 8>), g3, dim3(BlkGeom<8>::threads), 0, st, p4, a, bk, out); \
    else                                                                                                    \
      hipLaunchKernelGGL((bev_blk_strip_kernel<L, F, 4>), g3, dim3(BlkGeom<4>::threads), 0, st, p4, a, bk, out); \
  } while (0)
      switch (out_layout) {
        case SFA_BEV_NCHW3_F32:
          if (flip) SFA_BEV_BLK(SFA_BEV_NCHW3_F32, true); else SFA_BEV_BLK(SFA_BEV_NCHW3_F32, false);
          break;
        case SFA_BEV_NCHW3_F64:
          if (flip) SFA_BEV_BLK(SFA_BEV_NCHW3_F64, true); else SFA_BEV_BLK(SFA_BEV_NCHW3_F64, false);
          break;
        default:
          if (flip) SFA_BEV_BLK(SFA_BEV_NHWC4_F32, true); else SFA_BEV_BLK(SFA_BEV_NHWC4_F32, false);
      }
#undef SFA_BEV_BLK
      SFA_LAUNCH_CHECK();
      return SFA_OK;
    }
  }
  // binned path (round 2) when forced or when the blocked regions do not fit
  const size_t bin_bytes = align_up((size_t)cap * kStrips * sizeof(unsigned), 256);
  const size_t binned_bytes = bev_atomic_bytes(cap);  // the binned path's region
  const int64_t total = frame_offsets[batch] - frame_offsets[0];
  if (!force_atomic && 3 * bin_bytes < binned_bytes &&
      (uint64_t)total <= (uint64_t)((binned_bytes - 3 * bin_bytes) / sizeof(uint4)) && total < (int64_t)0xffffffff) {
    char* sb = reinterpret_cast<char*>(scratch) + bev_atomic_bytes(cap);
    BinScratch bs;
    bs.count = reinterpret_cast<unsigned*>(sb);
    bs.offset = reinterpret_cast<unsigned*>(sb + bin_bytes);
    bs.cursor = reinterpret_cast<unsigned*>(sb + 2 * bin_bytes);
    bs.rec = reinterpret_cast<uint4*>(sb + 3 * bin_bytes);
    if (max_n > 0) {
      dim3 g1((unsigned)((max_n + 256 * kBinPPT - 1) / (256 * kBinPPT)), batch);
      if (flags == SFA_BEV_RAW)
        hipLaunchKernelGGL(bev_bin_count_kernel<true>, g1, dim3(256), 0, st, p4, a, bs);
      else
        hipLaunchKernelGGL(bev_bin_count_kernel<false>, g1, dim3(256), 0, st, p4, a, bs);
      SFA_LAUNCH_CHECK();
      hipLaunchKernelGGL(bev_bin_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, bs, batch);
      SFA_LAUNCH_CHECK();
      if (flags == SFA_BEV_RAW)
        hipLaunchKernelGGL(bev_bin_kernel<true>, g1, dim3(256), 0, st, p4, a, bs);
      else
        hipLaunchKernelGGL(bev_bin_kernel<false>, g1, dim3(256), 0, st, p4, a, bs);
      SFA_LAUNCH_CHECK();
    }
    dim3 g3(kStrips, batch);
#define SFA_BEV_STRIP(L, F) \
  hipLaunchKernelGGL((bev_strip_kernel<L, F>), g3, dim3(kStripThreads), 0, st, p4, a, bs, out)
    switch (out_layout) {
      case SFA_BEV_NCHW3_F32:
        if (flip) SFA_BEV_STRIP(SFA_BEV_NCHW3_F32, true); else SFA_BEV_STRIP(SFA_BEV_NCHW3_F32, false);
        break;
      case SFA_BEV_NCHW3_F64:
        if (flip) SFA_BEV_STRIP(SFA_BEV_NCHW3_F64, true); else SFA_BEV_STRIP(SFA_BEV_NCHW3_F64, false);
        break;
      default:
        if (flip) SFA_BEV_STRIP(SFA_BEV_NHWC4_F32, true); else SFA_BEV_STRIP(SFA_BEV_NHWC4_F32, false);
    }
#undef SFA_BEV_STRIP
    SFA_LAUNCH_CHECK();
    return SFA_OK;
  }
  if (max_n > 0) {
    dim3 g1((unsigned)((max_n + 255) / 256), batch);
    if (flags == SFA_BEV_RAW)
      hipLaunchKernelGGL(bev_scatter_kernel<true>, g1, dim3(256), 0, st, p4, a, keys, counts);
    else
      hipLaunchKernelGGL(bev_scatter_kernel<false>, g1, dim3(256), 0, st, p4, a, keys, counts);
    SFA_LAUNCH_CHECK();
  }
  dim3 g2((unsigned)ceil_div(kBevCells, 256), batch);
#define SFA_BEV_GATHER(L, F) \
  hipLaunchKernelGGL((bev_gather_kernel<L, F>), g2, dim3(256), 0, st, p4, a, keys, counts, out)
  switch (out_layout) {
    case SFA_BEV_NCHW3_F32:
      if (flip) SFA_BEV_GATHER(SFA_BEV_NCHW3_F32, true); else SFA_BEV_GATHER(SFA_BEV_NCHW3_F32, false);
      break;
    case SFA_BEV_NCHW3_F64:
      if (flip) SFA_BEV_GATHER(SFA_BEV_NCHW3_F64, true); else SFA_BEV_GATHER(SFA_BEV_NCHW3_F64, false);
      break;
    default:
      if (flip) SFA_BEV_GATHER(SFA_BEV_NHWC4_F32, true); else SFA_BEV_GATHER(SFA_BEV_NHWC4_F32, false);
  }
#undef SFA_BEV_GATHER
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

// ---------------------------------------------------------------- filter --
// get_filtered_lidar (kitti_data_utils.py:228-251) as an order-preserving stream
// compaction: per-block keep counts -> one-block exclusive scan -> scatter with
// an in-block scan over contiguous per-thread ranges.
namespace sfa {

constexpr int kFiltThreads = 256;
constexpr int kFiltItems = 8;
constexpr int kFiltChunk = kFiltThreads * kFiltItems;

struct FiltArgs {
  float minX, maxX, minY, maxY, minZ, maxZ;
};

__device__ __forceinline__ bool keep_point(const float4& p, const FiltArgs& f) {
  return p.x >= f.minX && p.x <= f.maxX && p.y >= f.minY && p.y <= f.maxY && p.z >= f.minZ &&
         p.z <= f.maxZ;
}

__device__ int block_scan256(int v, int* sh /*[4]*/, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  int before = 0;
  for (int w = 0; w < wave; ++w) before += sh[w];
  *total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return before + x - v;
}

__global__ void __launch_bounds__(kFiltThreads) filter_count_kernel(const float4* __restrict__ pts,
                                                                    long long n, FiltArgs f,
                                                                    int* __restrict__ bcount) {
  __shared__ int sh[4];
  const long long base = (long long)blockIdx.x * kFiltChunk + (long long)threadIdx.x * kFiltItems;
  int c = 0;
#pragma unroll
  for (int j = 0; j < kFiltItems; ++j)
    if (base + j < n) c += keep_point(pts[base + j], f);
  int total;
  block_scan256(c, sh, &total);
  if (threadIdx.x == 0) bcount[blockIdx.x] = total;
}

__global__ void __launch_bounds__(1024) filter_scan_kernel(int* __restrict__ bcount, int nb,
                                                           long long* __restrict__ out_n) {
  __shared__ int wsum[16];
  __shared__ long long carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int base = 0; base < nb; base += 1024) {
    const int i = base + threadIdx.x;
    const int v = i < nb ? bcount[i] : 0;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int before = 0;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    int tot = 0;
    for (int w = 0; w < 16; ++w) tot += wsum[w];
    if (i < nb) bcount[i] = (int)(carry + before + x - v);
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *out_n = carry;
}

__global__ void __launch_bounds__(kFiltThreads) filter_scatter_kernel(
    const float4* __restrict__ pts, long long n, FiltArgs f, const int* __restrict__ boff,
    float4* __restrict__ out) {
  __shared__ int sh[4];
  const long long base = (long long)blockIdx.x * kFiltChunk + (long long)threadIdx.x * kFiltItems;
  float4 v[kFiltItems];
  bool k[kFiltItems];
  int c = 0;
#pragma unroll
  for (int j = 0; j < kFiltItems; ++j) {
    k[j] = false;
    if (base + j < n) {
      v[j] = pts[base + j];
      k[j] = keep_point(v[j], f);
    }
    c += k[j];
  }
  int total;
  int pos = boff[blockIdx.x] + block_scan256(c, sh, &total);
#pragma unroll
  for (int j = 0; j < kFiltItems; ++j)
    if (k[j]) {
      float4 q = v[j];
      q.z = __fsub_rn(q.z, f.minZ);  // :241
      out[pos++] = q;
    }
}

}  // namespace sfa

extern "C" size_t sfa_filter_scratch_size(int64_t n_points) {
  const long long nb = (n_points + kFiltChunk - 1) / kFiltChunk;
  return align_up((size_t)(nb > 0 ? nb : 1) * sizeof(int), 256) + 256;
}

extern "C" int sfa_filter_points(const float* points, int64_t n_points, const double* boundary,
                                 float* out, int64_t* out_count, void* scratch,
                                 size_t scratch_bytes, void* stream) {
  SFA_CHECK_ARG(n_points >= 0 && boundary && out_count && scratch, "filter: bad arguments");
  SFA_CHECK_ARG(n_points == 0 || (points && out), "filter: null points");
  SFA_CHECK_ARG(n_points < (1ll << 31) * (long long)kFiltChunk / 4, "filter: too many points");
  if (scratch_bytes < sfa_filter_scratch_size(n_points)) {
    set_error("filter: scratch too small");
    return SFA_E_WORKSPACE;
  }
  FiltArgs f{(float)boundary[0], (float)boundary[1], (float)boundary[2],
             (float)boundary[3], (float)boundary[4], (float)boundary[5]};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nb = (int)((n_points + kFiltChunk - 1) / kFiltChunk);
  int* bcount = reinterpret_cast<int*>(scratch);
  const float4* p4 = reinterpret_cast<const float4*>(points);
  if (nb == 0) {
    return launch_zero_words(out_count, sizeof(int64_t), st);  // a kernel node, not a memset (aux_kernels.h)
  }
  hipLaunchKernelGGL(filter_count_kernel, dim3(nb), dim3(kFiltThreads), 0, st, p4,
                     (long long)n_points, f, bcount);
  SFA_LAUNCH_CHECK();
  hipLaunchKernelGGL(filter_scan_kernel, dim3(1), dim3(1024), 0, st, bcount, nb,
                     reinterpret_cast<long long*>(out_count));
  SFA_LAUNCH_CHECK();
  hipLaunchKernelGGL(filter_scatter_kernel, dim3(nb), dim3(kFiltThreads), 0, st, p4,
                     (long long)n_points, f, bcount, reinterpret_cast<float4*>(out));
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}
