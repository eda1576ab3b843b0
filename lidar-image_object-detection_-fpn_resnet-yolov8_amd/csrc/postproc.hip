// Post-processing on device: decoded detections -> per-class rows
// (evaluation_utils.py:112-163) -> metres (:177-193) -> camera image boxes
// (test6.py:129-187 + transformation.py:99-107), so the detections reach the fusion
// kernel without a device->host hop.
//
// The work is a few hundred rows per batch: one workgroup, one wave per frame, rows
// compacted with ballots in the reference's order (class-major, decode order inside a
// class).  Output offsets need every frame's count first, so each kernel runs its
// frames twice: pass 0 counts (lane 0 stores the count in out_offsets[b + 1]), the
// block scans the counts in place, pass 1 recomputes and writes.  Recomputing ~K rows
// is cheaper than a second launch.
//
// Arithmetic follows the reference's dtypes exactly and is built with
// -ffp-contract=off (plus the pragma): an FMA in `a / b * c + d` or in a dot product
// would change the last bit of f32 post_processing outputs.
#include <math.h>

#include "common.h"

#pragma clang fp contract(off)

namespace sfa {

namespace {

constexpr int kWaves = 16;  // frames in flight per pass

__device__ __forceinline__ unsigned long long below_mask(int lane) {
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Exclusive scan in place: off[0] = 0, off[b + 1] = count of frame b on entry,
// prefix sums on exit.  Called by every thread of the block.
__device__ void block_scan_counts(int32_t* off, int batch) {
  __syncthreads();
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int carry = 0;
    for (int c0 = 0; c0 < batch; c0 += 64) {
      const int b = c0 + lane;
      int v = b < batch ? off[b + 1] : 0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
      }
      if (b < batch) off[b + 1] = carry + v;
      carry += __shfl(v, 63, 64);
    }
    if (lane == 0) off[0] = 0;
  }
  __syncthreads();
}

struct PostRow {
  float pred[8];
  double real[8];
};

// evaluation_utils.py:136-145 (f32) then :182-191 (f32 or f64 per p.arith)
__device__ __forceinline__ PostRow post_row(const float* d, int cls, const sfa_post_params& p) {
  PostRow r;
  const float down = (float)p.down_ratio;
  r.pred[0] = d[0];
  r.pred[1] = d[1] * down;
  r.pred[2] = d[2] * down;
  r.pred[3] = d[3];
  r.pred[4] = d[4];
  r.pred[5] = d[5] / (float)p.bound_y * (float)p.bev_w;
  r.pred[6] = d[6] / (float)p.bound_x * (float)p.bev_h;
  r.pred[7] = (float)atan2((double)d[7], (double)d[8]);  // get_yaw, :108-109
  const float _x = r.pred[1], _y = r.pred[2], _z = r.pred[3], _w = r.pred[5], _l = r.pred[6];
  r.real[0] = (double)cls;
  if (p.arith == SFA_REAL_F32) {  // numpy >= 2: f32 scalar (op) Python number stays f32
    r.real[1] = (double)(_y / (float)p.bev_h * (float)p.bound_x + (float)p.min_x);
    r.real[2] = (double)(_x / (float)p.bev_w * (float)p.bound_y + (float)p.min_y);
    r.real[3] = (double)(_z + (float)p.min_z);
    r.real[5] = (double)(_w / (float)p.bev_w * (float)p.bound_y);
    r.real[6] = (double)(_l / (float)p.bev_h * (float)p.bound_x);
  } else {  // numpy 1.x: promoted to f64
    r.real[1] = (double)_y / (double)p.bev_h * p.bound_x + p.min_x;
    r.real[2] = (double)_x / (double)p.bev_w * p.bound_y + p.min_y;
    r.real[3] = (double)_z + p.min_z;
    r.real[5] = (double)_w / (double)p.bev_w * p.bound_y;
    r.real[6] = (double)_l / (double)p.bev_h * p.bound_x;
  }
  r.real[4] = (double)r.pred[4];
  r.real[7] = (double)(-r.pred[7]);
  return r;
}

__global__ void __launch_bounds__(64 * kWaves)
    post_process_kernel(const float* __restrict__ dets, int batch, int K, sfa_post_params p,
                        float* __restrict__ out_preds, double* __restrict__ out_real,
                        int32_t* __restrict__ off) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int pass = 0; pass < 2; ++pass) {
    for (int b = wave; b < batch; b += kWaves) {
      const float* d = dets + (size_t)b * K * 10;
      const int base = pass ? off[b] : 0;
      int n = 0;
      for (int j = 0; j < p.num_classes; ++j) {
        for (int c0 = 0; c0 < K; c0 += 64) {
          const int i = c0 + lane;
          bool keep = false;
          if (i < K) keep = d[i * 10 + 9] == (float)j && d[i * 10] > p.peak_thresh;
          const unsigned long long m = __ballot(keep);
          if (pass && keep) {
            const int pos = base + n + __popcll(m & below_mask(lane));
            const PostRow r = post_row(d + i * 10, j, p);
#pragma unroll
            for (int c = 0; c < 8; ++c) {
              out_preds[(size_t)pos * 8 + c] = r.pred[c];
              out_real[(size_t)pos * 8 + c] = r.real[c];
            }
          }
          n += __popcll(m);
        }
      }
      if (!pass && lane == 0) off[b + 1] = n;
    }
    if (!pass) block_scan_counts(off, batch);
  }
}

// test6.py:143-182 for one real row; false when the box is not kept.
__device__ __forceinline__ bool project_row(const double* rr, const sfa_calib& c, double ext[4]) {
  const double x = rr[1], y = rr[2], z = rr[3], h = rr[4], w = rr[5], l = rr[6], rz = rr[7];
  // lidar_to_camera (transformation.py:50-59): V2C @ [x, y, z, 1], then R0 @ .
  double cam[3], rect[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double s = c.V2C[i * 4] * x;
    s = s + c.V2C[i * 4 + 1] * y;
    s = s + c.V2C[i * 4 + 2] * z;
    s = s + c.V2C[i * 4 + 3] * 1.0;
    cam[i] = s;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double s = c.R0[i * 3] * cam[0];
    s = s + c.R0[i * 3 + 1] * cam[1];
    s = s + c.R0[i * 3 + 2] * cam[2];
    rect[i] = s;
  }
  const double ry = -rz - M_PI / 2;  // transformation.py:104
  double sn, cs;
  sincos(ry, &sn, &cs);
  const double hl = l / 2, hw = w / 2;
  double mnx = 0, mxx = 0, mny = 0, mxy = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const double cx = (k == 0 || k == 1 || k == 4 || k == 5) ? -hl : hl;   // test6.py:151
    const double cy = k < 4 ? 0.0 : -h;                                     // :152
    const double cz = (k == 0 || k == 3 || k == 4 || k == 7) ? -hw : hw;   // :153
    const double X = cs * cx + sn * cz + rect[0];
    const double Y = cy + rect[1];
    const double Z = -sn * cx + cs * cz + rect[2];
    double pu = c.P2[0] * X, pv = c.P2[4] * X, pw = c.P2[8] * X;
    pu = pu + c.P2[1] * Y;
    pv = pv + c.P2[5] * Y;
    pw = pw + c.P2[9] * Y;
    pu = pu + c.P2[2] * Z;
    pv = pv + c.P2[6] * Z;
    pw = pw + c.P2[10] * Z;
    pu = pu + c.P2[3] * 1.0;
    pv = pv + c.P2[7] * 1.0;
    pw = pw + c.P2[11] * 1.0;
    const double u = pu / pw, v = pv / pw;
    if (k == 0) {
      mnx = mxx = u;
      mny = mxy = v;
    } else {  // np.min / np.max propagate NaN
      mnx = (u < mnx || isnan(u)) && !isnan(mnx) ? u : mnx;
      mxx = (u > mxx || isnan(u)) && !isnan(mxx) ? u : mxx;
      mny = (v < mny || isnan(v)) && !isnan(mny) ? v : mny;
      mxy = (v > mxy || isnan(v)) && !isnan(mxy) ? v : mxy;
    }
  }
  // Python max(0, v) keeps v only when v > 0; min(img, v) only when v < img (:176-179)
  mnx = mnx > 0 ? mnx : 0.0;
  mny = mny > 0 ? mny : 0.0;
  mxx = mxx < (double)c.img_w ? mxx : (double)c.img_w;
  mxy = mxy < (double)c.img_h ? mxy : (double)c.img_h;
  ext[0] = mnx;
  ext[1] = mny;
  ext[2] = mxx;
  ext[3] = mxy;
  return mxx > mnx && mxy > mny;  // :181
}

__global__ void __launch_bounds__(64 * kWaves)
    project_boxes_kernel(const double* __restrict__ real, const float* __restrict__ preds,
                         const int32_t* __restrict__ in_off, int batch,
                         const sfa_calib* __restrict__ calib, sfa_project_params p,
                         int4* __restrict__ out_boxes, double* __restrict__ out_conf,
                         int32_t* __restrict__ out_row, double* __restrict__ out_ext,
                         int32_t* __restrict__ off) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int pass = 0; pass < 2; ++pass) {
    for (int b = wave; b < batch; b += kWaves) {
      const sfa_calib& c = calib[p.calib_per_frame ? b : 0];
      const int r0 = in_off[b], nr = in_off[b + 1] - r0;
      const int base = pass ? off[b] : 0;
      int n = 0;
      for (int c0 = 0; c0 < nr; c0 += 64) {
        const int i = c0 + lane;
        bool keep = false;
        double conf = 0, ext[4];
        if (i < nr) {
          const double* rr = real + (size_t)(r0 + i) * 8;
          conf = p.conf_source == SFA_CONF_SCORE ? (double)preds[(size_t)(r0 + i) * 8] : rr[0];
          keep = conf >= p.conf_min && project_row(rr, c, ext);  // test6.py:138-140
        }
        const unsigned long long m = __ballot(keep);
        if (pass && keep) {
          const int pos = base + n + __popcll(m & below_mask(lane));
          // int() truncates toward zero; 0 <= min < max <= img here, so it fits
          out_boxes[pos] = make_int4((int)ext[0], (int)ext[1], (int)(ext[2] - ext[0]),
                                     (int)(ext[3] - ext[1]));
          out_conf[pos] = conf;
          out_row[pos] = i;
          if (out_ext) {
#pragma unroll
            for (int e = 0; e < 4; ++e) out_ext[(size_t)pos * 4 + e] = ext[e];
          }
        }
        n += __popcll(m);
      }
      if (!pass && lane == 0) off[b + 1] = n;
    }
    if (!pass) block_scan_counts(off, batch);
  }
}

}  // namespace

}  // namespace sfa

using namespace sfa;

extern "C" int sfa_post_process(const float* dets, int batch, int K, const sfa_post_params* params,
                                float* out_preds, double* out_real, int32_t* out_offsets,
                                void* stream) {
  SFA_CHECK_ARG(params && batch >= 0 && K >= 0 && out_offsets, "post_process: bad arguments");
  SFA_CHECK_ARG(batch * (long long)K == 0 || (dets && out_preds && out_real),
                "post_process: null buffer");
  SFA_CHECK_ARG(params->num_classes >= 0 && params->bev_h > 0 && params->bev_w > 0 &&
                    params->arith >= SFA_REAL_F32 && params->arith <= SFA_REAL_F64,
                "post_process: bad params");
  hipLaunchKernelGGL(post_process_kernel, dim3(1), dim3(64 * kWaves), 0,
                     reinterpret_cast<hipStream_t>(stream), dets, batch, K, *params, out_preds,
                     out_real, out_offsets);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

extern "C" int sfa_project_boxes(const double* real, const float* preds, const int32_t* offsets,
                                 int batch, const sfa_calib* calib,
                                 const sfa_project_params* params, int32_t* out_boxes,
                                 double* out_conf, int32_t* out_row, double* out_extent,
                                 int32_t* out_offsets, void* stream) {
  SFA_CHECK_ARG(params && batch >= 0 && offsets && out_offsets && calib,
                "project_boxes: bad arguments");
  SFA_CHECK_ARG(real && out_boxes && out_conf && out_row, "project_boxes: null buffer");
  SFA_CHECK_ARG(params->conf_source == SFA_CONF_CLASS_ID ||
                    (params->conf_source == SFA_CONF_SCORE && preds),
                "project_boxes: SFA_CONF_SCORE needs preds");
  hipLaunchKernelGGL(project_boxes_kernel, dim3(1), dim3(64 * kWaves), 0,
                     reinterpret_cast<hipStream_t>(stream), real, preds, offsets, batch, calib,
                     *params, reinterpret_cast<int4*>(out_boxes), out_conf, out_row, out_extent,
                     out_offsets);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}
