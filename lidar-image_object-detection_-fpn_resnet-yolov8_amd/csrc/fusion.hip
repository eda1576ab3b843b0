// Camera-LiDAR late fusion + greedy NMS (BASELINE configs[4]).
//
// Reference (host Python, O(n^2) loops over tens of boxes per frame):
//   test6.py:76-101   calculate_iou          [x, y, w, h] ints, IoU in f64
//   test6.py:310-348  create_fused_detections_wrapper  conf >= threshold filter
//   test6.py:231-308  bayesian_inspired_fuse_overlapping_detections (inverse-variance)
//   test5.py:213-282  fuse_overlapping_detections (confidence-weighted average)
//   test6.py:104-126  apply_nms_to_fused_detections (stable sort by conf, greedy, IoU >)
//
// One 64-lane wavefront per frame: the association is sequential over YOLO boxes by
// definition (each takes the best still-unmatched SFA box), so every step is a
// wave-wide IoU sweep + shuffle arg-max (ties -> lower SFA index, as the strict '>'
// of the reference loop); the NMS is a wave-parallel rank sort followed by a greedy
// sweep whose per-candidate test (IoU against every kept box) is a wave vote.
// Arithmetic is IEEE f64 with no FMA contraction (pragma below + -ffp-contract=off), so every
// box, confidence and keep decision is bit-identical to the Python reference.
#include "common.h"

// Plain f64 operators under contract(off): hipcc's default -ffp-contract=fast would
// fuse m1*i1 + m2*i2 into an FMA (HIP's __dadd_rn/__dmul_rn are plain operators in a
// header, so they are contracted too), and a fused coordinate that lands near an
// integer would then truncate differently from Python.
#pragma clang fp contract(off)

namespace sfa {

constexpr int kFuseMax = 512;  // boxes per side per frame

struct FuseArgs {
  double conf_thr, fusion_iou, nms_thr;
  int mode, apply_nms;
};

__device__ __forceinline__ double box_iou(int4 a, int4 b) {
  const long long xl = max(a.x, b.x), yt = max(a.y, b.y);
  const long long xr = min((long long)a.x + a.z, (long long)b.x + b.z);
  const long long yb = min((long long)a.y + a.w, (long long)b.y + b.w);
  if (xr < xl || yb < yt) return 0.0;
  const long long inter = (xr - xl) * (yb - yt);
  const long long uni = (long long)a.z * a.w + (long long)b.z * b.w - inter;
  return uni > 0 ? (double)inter / (double)uni : 0.0;
}

__device__ __forceinline__ double conf_to_var(double c, double vmax) {  // test6.py:212-215
  return c < 0.1 ? (vmax * 100.0)
                 : vmax * ((1.0 - c) / (c + 0.01));
}

__device__ __forceinline__ double gauss_mean(double m1, double v1, double m2, double v2) {
  v1 = v1 >= 1e-6 ? v1 : 1e-6;  // max(var, epsilon), test6.py:219-221
  v2 = v2 >= 1e-6 ? v2 : 1e-6;
  const double i1 = (1.0 / v1), i2 = (1.0 / v2);
  const double a = m1 * i1, b = m2 * i2;
  return (a + b) / (i1 + i2);
}

__device__ __forceinline__ int py_int(double x) { return (int)(long long)x; }  // trunc to 0

__device__ __forceinline__ unsigned long long lanes_below() {
  const int lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

__global__ void __launch_bounds__(64) fuse_kernel(
    const int4* __restrict__ ybox_in, const double* __restrict__ yconf_in,
    const int* __restrict__ ycls_in, const int* __restrict__ yoff, const int4* __restrict__ sbox_in,
    const double* __restrict__ sconf_in, const int* __restrict__ soff, FuseArgs p,
    int4* __restrict__ obox, double* __restrict__ oconf, int* __restrict__ ocls,
    int* __restrict__ osrc, int* __restrict__ oorig, int* __restrict__ omatch,
    int* __restrict__ ocount, int* __restrict__ okeep, int* __restrict__ okeep_count) {
  __shared__ int4 ybox[kFuseMax], sbox[kFuseMax], fbox[2 * kFuseMax];
  __shared__ double yconf[kFuseMax], sconf[kFuseMax], fconf[2 * kFuseMax];
  __shared__ int ycls[kFuseMax], smatched[kFuseMax], fcls[2 * kFuseMax], fsrc[2 * kFuseMax];
  __shared__ int order[2 * kFuseMax], keep[2 * kFuseMax];
  __shared__ int yidx[kFuseMax], sidx[kFuseMax], forig[2 * kFuseMax], fmatch[2 * kFuseMax];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int y0 = yoff[b], ny = yoff[b + 1] - y0;
  const int s0 = soff[b], ns = soff[b + 1] - s0;
  const int base = y0 + s0;
  if (ny > kFuseMax || ns > kFuseMax || ny < 0 || ns < 0) {  // frame too large: flagged, untouched
    if (lane == 0) {
      ocount[b] = -1;
      if (p.apply_nms) okeep_count[b] = -1;
    }
    return;
  }

  // conf >= threshold, order preserved (create_fused_detections_wrapper, test6.py:320-340)
  int nyf = 0;
  for (int c0 = 0; c0 < ny; c0 += 64) {
    const int i = c0 + lane;
    const bool k = i < ny && yconf_in[y0 + i] >= p.conf_thr;
    const unsigned long long m = __ballot(k);
    if (k) {
      const int pos = nyf + __popcll(m & lanes_below());
      ybox[pos] = ybox_in[y0 + i];
      yconf[pos] = yconf_in[y0 + i];
      ycls[pos] = ycls_in[y0 + i];
      yidx[pos] = i;
    }
    nyf += __popcll(m);
  }
  int nsf = 0;
  for (int c0 = 0; c0 < ns; c0 += 64) {
    const int i = c0 + lane;
    const bool k = i < ns && sconf_in[s0 + i] >= p.conf_thr;
    const unsigned long long m = __ballot(k);
    if (k) {
      const int pos = nsf + __popcll(m & lanes_below());
      sbox[pos] = sbox_in[s0 + i];
      sconf[pos] = sconf_in[s0 + i];
      smatched[pos] = 0;
      sidx[pos] = i;
    }
    nsf += __popcll(m);
  }
  __syncthreads();

  // association + fusion, sequential over the YOLO detections (test6.py:240-300)
  for (int i = 0; i < nyf; ++i) {
    const int4 yb = ybox[i];
    double best = 0.0;
    int bj = 0x7fffffff;
    for (int j = lane; j < nsf; j += 64) {
      if (smatched[j]) continue;
      const double v = box_iou(yb, sbox[j]);
      if (v > 0.0 && v >= p.fusion_iou && (v > best || (v == best && j < bj))) {
        best = v;
        bj = j;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double ob = __shfl_xor(best, o, 64);
      const int oj = __shfl_xor(bj, o, 64);
      if (ob > best || (ob == best && oj < bj)) {
        best = ob;
        bj = oj;
      }
    }
    if (lane == 0) {
      const double yc = yconf[i];
      if (bj != 0x7fffffff) {
        const int4 sb = sbox[bj];
        const double sc = sconf[bj];
        int4 f;
        if (p.mode == SFA_FUSE_BAYES) {
          f.x = py_int(gauss_mean(yb.x, conf_to_var(yc, 100.0), sb.x, conf_to_var(sc, 100.0)));
          f.y = py_int(gauss_mean(yb.y, conf_to_var(yc, 100.0), sb.y, conf_to_var(sc, 100.0)));
          f.z = py_int(gauss_mean(yb.z, conf_to_var(yc, 50.0), sb.z, conf_to_var(sc, 50.0)));
          f.w = py_int(gauss_mean(yb.w, conf_to_var(yc, 50.0), sb.w, conf_to_var(sc, 50.0)));
        } else {  // test5.py:246-260
          const double tot = (yc + sc);
          const double wy = tot == 0.0 ? 0.5 : (yc / tot);
          const double ws = tot == 0.0 ? 0.5 : (sc / tot);
          { const double a = wy * yb.x, b = ws * sb.x; f.x = py_int(a + b); }
          { const double a = wy * yb.y, b = ws * sb.y; f.y = py_int(a + b); }
          { const double a = wy * yb.z, b = ws * sb.z; f.z = py_int(a + b); }
          { const double a = wy * yb.w, b = ws * sb.w; f.w = py_int(a + b); }
        }
        fbox[i] = f;
        fconf[i] = yc >= sc ? yc : sc;  // max(yolo_conf, sfa3d_conf)
        fcls[i] = ycls[i];
        fsrc[i] = SFA_FUSED;
        forig[i] = yidx[i];
        fmatch[i] = sidx[bj];
        smatched[bj] = 1;
      } else {
        fbox[i] = yb;
        fconf[i] = yc;
        fcls[i] = ycls[i];
        fsrc[i] = SFA_SRC_YOLO;
        forig[i] = yidx[i];
        fmatch[i] = -1;
      }
    }
    __syncthreads();
  }
  // unmatched SFA detections, in order (test6.py:303-306); class id 0 ('car', :337)
  int nf = nyf;
  for (int c0 = 0; c0 < nsf; c0 += 64) {
    const int j = c0 + lane;
    const bool k = j < nsf && !smatched[j];
    const unsigned long long m = __ballot(k);
    if (k) {
      const int pos = nf + __popcll(m & lanes_below());
      fbox[pos] = sbox[j];
      fconf[pos] = sconf[j];
      fcls[pos] = 0;
      fsrc[pos] = SFA_SRC_LIDAR;
      forig[pos] = sidx[j];
      fmatch[pos] = -1;
    }
    nf += __popcll(m);
  }
  __syncthreads();
  for (int i = lane; i < nf; i += 64) {
    obox[base + i] = fbox[i];
    oconf[base + i] = fconf[i];
    ocls[base + i] = fcls[i];
    osrc[base + i] = fsrc[i];
    if (oorig) oorig[base + i] = forig[i];
    if (omatch) omatch[base + i] = fmatch[i];
  }
  if (lane == 0) ocount[b] = nf;
  if (!p.apply_nms) return;

  // NMS (test6.py:104-126): stable descending sort = rank by (conf desc, index asc)
  for (int i = lane; i < nf; i += 64) {
    const double c = fconf[i];
    int r = 0;
    for (int j = 0; j < nf; ++j) r += (fconf[j] > c) || (fconf[j] == c && j < i);
    order[r] = i;
  }
  __syncthreads();
  int nk = 0;
  for (int k = 0; k < nf; ++k) {
    const int c = order[k];
    const int4 cb = fbox[c];
    bool sup = false;
    for (int t = lane; t < nk; t += 64) sup |= box_iou(cb, fbox[keep[t]]) > p.nms_thr;
    if (!__any(sup)) {
      if (lane == 0) keep[nk] = c;
      ++nk;
      __syncthreads();
    }
  }
  for (int t = lane; t < nk; t += 64) okeep[base + t] = keep[t];
  if (lane == 0) okeep_count[b] = nk;
}

// Gaussian soft-NMS (reference README.md:250-261 gaussian_nms; the only definition the
// reference has, see SURVEY.md's north-star note): for i in order, every later detection j
// decays, conf_j *= exp(-iou(i, j)^2 / sigma) — no re-sorting, no threshold, boxes unchanged.
// conf_j's factors are therefore applied in i = 0 .. j-1 order, which lane j reproduces exactly
// (f64, no contraction); exp is the device's f64 exp (numpy's np.exp may differ in the last
// bit, so the confidences are pinned to ~1e-15 relative, not bitwise). One wave per frame.
__global__ void __launch_bounds__(256) gaussian_nms_kernel(int batch, const int4* __restrict__ boxes,
                                                           double* __restrict__ conf,
                                                           const int32_t* __restrict__ starts,
                                                           const int32_t* __restrict__ counts,
                                                           double sigma) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= batch) return;
  const int n = counts[b], s0 = starts[b];
  for (int j = lane; j < n; j += 64) {
    const int4 bj = boxes[s0 + j];
    double c = conf[s0 + j];
    for (int i = 0; i < j; ++i) {
      const double iou = box_iou(boxes[s0 + i], bj);  // calculate_iou(det_i, det_j), symmetric
      c = c * exp(-(iou * iou) / sigma);
    }
    conf[s0 + j] = c;
  }
}

__global__ void __launch_bounds__(256) iou_matrix_kernel(const int4* __restrict__ a, int na,
                                                         const int4* __restrict__ b, int nb,
                                                         double* __restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)na * nb) return;
  const int i = (int)(t / nb), j = (int)(t - (long long)i * nb);
  out[t] = box_iou(a[i], b[j]);
}

}  // namespace sfa

using namespace sfa;

extern "C" int sfa_iou_matrix(const int32_t* boxes_a, int na, const int32_t* boxes_b, int nb,
                              double* out, void* stream) {
  SFA_CHECK_ARG(na >= 0 && nb >= 0 && (na == 0 || boxes_a) && (nb == 0 || boxes_b) &&
                    (na * (long long)nb == 0 || out),
                "iou_matrix: bad arguments");
  const long long n = (long long)na * nb;
  if (n == 0) return SFA_OK;
  hipLaunchKernelGGL(iou_matrix_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const int4*>(boxes_a),
                     na, reinterpret_cast<const int4*>(boxes_b), nb, out);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

extern "C" int sfa_fuse_detections(int batch, const int32_t* yolo_boxes, const double* yolo_conf,
                                   const int32_t* yolo_cls, const int32_t* yolo_offsets,
                                   const int32_t* sfa_boxes, const double* sfa_conf,
                                   const int32_t* sfa_offsets, const sfa_fusion_params* params,
                                   int32_t* out_boxes, double* out_conf, int32_t* out_cls,
                                   int32_t* out_src, int32_t* out_origin, int32_t* out_match,
                                   int32_t* out_count, int32_t* out_keep, int32_t* out_keep_count,
                                   void* stream) {
  SFA_CHECK_ARG(batch >= 1 && params && yolo_offsets && sfa_offsets, "fuse: bad arguments");
  SFA_CHECK_ARG(out_boxes && out_conf && out_cls && out_src && out_count, "fuse: null output");
  SFA_CHECK_ARG(!params->apply_nms || (out_keep && out_keep_count), "fuse: null NMS output");
  SFA_CHECK_ARG(params->mode == SFA_FUSE_BAYES || params->mode == SFA_FUSE_WEIGHTED,
                "fuse: bad mode %d", params->mode);
  FuseArgs a{params->conf_threshold, params->fusion_iou_threshold, params->nms_threshold,
             params->mode, params->apply_nms};
  hipLaunchKernelGGL(fuse_kernel, dim3(batch), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const int4*>(yolo_boxes), yolo_conf, yolo_cls, yolo_offsets,
                     reinterpret_cast<const int4*>(sfa_boxes), sfa_conf, sfa_offsets, a,
                     reinterpret_cast<int4*>(out_boxes), out_conf, out_cls, out_src, out_origin,
                     out_match, out_count, out_keep, out_keep_count);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}

extern "C" int sfa_gaussian_nms(int batch, const int32_t* boxes, double* conf, const int32_t* starts,
                                const int32_t* counts, double sigma, void* stream) {
  SFA_CHECK_ARG(batch >= 0 && (batch == 0 || (boxes && conf && starts && counts)), "gaussian_nms: bad arguments");
  SFA_CHECK_ARG(sigma > 0.0, "gaussian_nms: sigma must be > 0 (got %g)", sigma);
  if (batch == 0) return SFA_OK;
  hipLaunchKernelGGL(gaussian_nms_kernel, dim3((unsigned)((batch + 3) / 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), batch, reinterpret_cast<const int4*>(boxes), conf,
                     starts, counts, sigma);
  SFA_LAUNCH_CHECK();
  return SFA_OK;
}
