/*
 * sfa_hip.h — C ABI of the MI355X (gfx950) hot path of the SFA3D-style
 * FPN-ResNet-18 LiDAR detector: BEV voxelisation -> KFPN forward -> decode.
 *
 * Plain C: pointers, sizes and status codes only; no torch / C++ types.
 * Every entry point that touches the device takes the caller's hipStream_t
 * (passed as void*), never allocates, never synchronises, and is re-entrant
 * per stream; all buffers (including scratch/workspace) are owned by the
 * caller.  Return value: SFA_OK (0) or a negative SFA_E_* code, with a
 * human-readable reason in sfa_last_error_string() (thread-local).
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to the reference repository root).
 */
#ifndef SFA_HIP_H_
#define SFA_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFA_ABI_VERSION 2  /* 2: sfa_bev_voxelize takes scratch_bytes */

enum sfa_status {
  SFA_OK = 0,
  SFA_E_INVALID = -1,   /* bad argument / shape */
  SFA_E_UNSUPPORTED = -2, /* configuration the kernels do not cover */
  SFA_E_HIP = -3,       /* a HIP runtime call failed */
  SFA_E_WORKSPACE = -4  /* workspace / scratch too small */
};

int sfa_abi_version(void);
const char* sfa_last_error_string(void);

/* ------------------------------------------------------------------ BEV --
 * Replaces data_process/kitti_data_utils.py:228-251 get_filtered_lidar followed
 * by data_process/kitti_bev_utils.py:22-55 makeBEVMap, for a batch of frames.
 *
 * points          device, float32 [total_points][4] = x, y, z, intensity (raw,
 *                 unfiltered; the kernel applies the inclusive boundary test)
 * frame_offsets   HOST, int64 [batch + 1]; frame b = points[off[b], off[b+1])
 * batch           1 .. SFA_BEV_MAX_BATCH
 * boundary        HOST, double [6] = minX, maxX, minY, maxY, minZ, maxZ
 *                 (config/kitti_config.py:23-30)
 * flags           SFA_BEV_RAW: raw sweep in, the get_filtered_lidar box test and
 *                 z -= minZ are fused in (the fast path);
 *                 SFA_BEV_PREFILTERED: points already went through
 *                 get_filtered_lidar (makeBEVMap's own contract); no box test.
 * out_layout      SFA_BEV_NCHW3_F32  (B, 3, 608, 608) float32  (== .float() of the
 *                                    reference's float64 map, test.py:124)
 *                 SFA_BEV_NCHW3_F64  (B, 3, 608, 608) float64  (reference dtype)
 *                 SFA_BEV_NHWC4_F32  (B, 608, 608, 4) float32, channel 3 = 0
 *                                    (the model's input layout; no transpose)
 *                 | SFA_BEV_FLIP_HW: the map is written flipped in both spatial
 *                 dims (torch.flip(bev, [1, 2]), utils/demo_utils.py:110-111 — the
 *                 back view of demo_2_sides.py with boundary_back)
 * scratch         device, scratch_bytes >= sfa_bev_scratch_size(batch) bytes (else
 *                 SFA_E_WORKSPACE), ZERO on first use; every call leaves it zeroed again
 *                 except the record regions, which are written before they are read.  The
 *                 layout is set by the capacity (the largest batch scratch_bytes holds), not
 *                 by the call's batch, so calls of any batch may share one scratch.
 * Kernels: one pass bins every 1024 points of a frame by 4-row strips of the map into
 * the pass block's own record region + a per-strip table, then one block per (frame, strip)
 * reduces its runs in LDS, while the batch's regions fit the scratch (~277 k points per
 * frame; SFA_BEV_STRIP8: 8-row strips); SFA_BEV_FORCE_BINNED: round 2's count / scan / bin / strip form; otherwise (or with
 * SFA_BEV_FORCE_ATOMIC) device-scope atomics on a per-cell scratch.  All give the same bits.
 */
#define SFA_BEV_MAX_BATCH 64
enum sfa_bev_layout { SFA_BEV_NCHW3_F32 = 0, SFA_BEV_NCHW3_F64 = 1, SFA_BEV_NHWC4_F32 = 2 };
enum sfa_bev_flags {
  SFA_BEV_RAW = 0, SFA_BEV_PREFILTERED = 1, SFA_BEV_FLIP_HW = 2, SFA_BEV_FORCE_ATOMIC = 4,
  SFA_BEV_FORCE_BINNED = 8,  /* round 2's count / scan / bin / strip kernels (A/B) */
  SFA_BEV_STRIP8 = 16        /* the one-pass path with 8-row strips (round 3a; A/B) */
};

size_t sfa_bev_scratch_size(int batch);
int sfa_bev_voxelize(const float* points, const int64_t* frame_offsets, int batch,
                     const double* boundary, int flags, int out_layout, void* out, void* scratch,
                     size_t scratch_bytes, void* stream);

/* Replaces data_process/kitti_data_utils.py:228-251 get_filtered_lidar (labels=None):
 * order-preserving compaction of the points inside the inclusive box, with
 * z <- z - minZ.  points/out device float32 [n][4]; out must hold n points;
 * *out_count (DEVICE int64) receives the kept count.  scratch: device,
 * sfa_filter_scratch_size(n) bytes. */
size_t sfa_filter_scratch_size(int64_t n_points);
int sfa_filter_points(const float* points, int64_t n_points, const double* boundary, float* out,
                      int64_t* out_count, void* scratch, size_t scratch_bytes, void* stream);

/* ---------------------------------------------------------------- model --
 * Replaces models/model_utils.py:25-43 create_model -> models/fpn_resnet.py
 * get_pose_net(18, heads, 64) (:296-301) and PoseResNet.forward (:169-246).
 *
 * Architecture descriptor: resnet depth (18 only), head_conv (64 only) and the
 * heads in FORWARD order (the `heads` dict insertion order, fpn_resnet.py:220);
 * the state_dict registers them in sorted() order (fpn_resnet.py:135).
 */
#define SFA_MAX_HEADS 8
typedef struct sfa_arch {
  int num_layers;                 /* 18 */
  int head_conv;                  /* 64 */
  int num_heads;                  /* 1 .. SFA_MAX_HEADS */
  int head_channels[SFA_MAX_HEADS]; /* 1 .. 4 each, forward order */
  char head_names[SFA_MAX_HEADS][32];
} sfa_arch;

/* Reference state_dict layout (186 entries for fpn_resnet_18 with 5 heads), in
 * nn.Module registration order.  shape is padded with 0s; ndim 0 = scalar. */
int sfa_state_count(const sfa_arch* arch);
int sfa_state_entry(const sfa_arch* arch, int index, char* name, int name_len, int64_t* shape4,
                    int* ndim);

/* Pack weights (host -> host): `state` = the float32 values of every
 * state_dict entry except *.num_batches_tracked, concatenated in
 * sfa_state_entry order.  BatchNorm (eps 1e-5) is folded into the preceding
 * convolution; conv weights are re-laid out OHWI / K-concatenated for the
 * implicit-GEMM kernels, each also stored as three bf16 terms for SFA_MATH_BF16X6 and,
 * scaled per output channel by a power of two, as two fp16 terms for SFA_MATH_FP16X3.
 * `packed` must hold sfa_packed_floats(arch) floats. */
size_t sfa_state_floats(const sfa_arch* arch);
size_t sfa_packed_floats(const sfa_arch* arch);
int sfa_pack_weights(const sfa_arch* arch, const float* state, size_t state_floats, float* packed);

/* A model handle references a device copy of the packed weights (caller-owned,
 * must outlive the handle).  No device memory is allocated.  The handle owns side
 * streams + events on the device current at creation: a forward on a stream of that
 * device runs the level-0 detection heads on a side stream (overlapping the rest of the FPN)
 * and the level-2 heads beside the level-1 heads, forked/joined by events, so HIP-graph capture of the
 * caller's stream records every branch; on another device everything stays on the caller's
 * stream. */
typedef struct sfa_model sfa_model;
int sfa_model_create(const sfa_arch* arch, const float* packed_device, sfa_model** out);
void sfa_model_destroy(sfa_model* model);

/* Side streams on (1, the default; env SFA_SIDE_STREAMS=0 at create time turns them off) or
 * off (0: every launch of the forward on the caller's stream).  Off destroys them (after their
 * last forward has finished), on creates them on the current device.  Every stream of a
 * process takes one of HIP's hardware queues (4 by default), so a caller running several
 * forwards in flight beside a copy stream turns them off (the KITTI .bin stream workload:
 * profiles/r02b_stream_side_streams.txt).  Not concurrently with a forward of this model.
 * No reference counterpart (measurement / scheduling). */
int sfa_model_set_side_streams(sfa_model* model, int on);

/* Arithmetic of the convolutions (all results are f32; every mode meets the parity
 * bar):
 *   SFA_MATH_FP16X3 (default) — operands scaled by powers of two (weights per output channel at
 *     pack time, activations per tensor and frame from the max |x| their producer records) and
 *     split into two fp16 terms (22 significand bits), the three significant products on
 *     fp16 MFMA with f32 accumulation: half the MFMA work of BF16X6 at the same accuracy
 *     class (max rel. logit error vs the reference ~3e-6); the scales never overflow fp16
 *     (scaled |x| < 2^14), and each frame is scaled by its own maxima (batch-invariant);
 *   SFA_MATH_BF16X6 — every f32 operand split into three bf16 terms, the six significant
 *     products on bf16 MFMA with f32 accumulation (full f32 exponent range, no scaling);
 *   SFA_MATH_F32 — v_mfma_f32_32x32x2_f32 (exact f32 FMA chains). */
enum sfa_math { SFA_MATH_F32 = 0, SFA_MATH_BF16X6 = 1, SFA_MATH_FP16X3 = 2 };
int sfa_model_set_math(sfa_model* model, int math);
int sfa_model_get_math(const sfa_model* model);

/* Kernel-choice options of a model handle (no reference counterpart: the equivalence tests and
 * A/B runs of the two forms each option selects).  Every option is a field of the handle, read by
 * the forward when it enqueues its launches (a captured graph keeps the choice of its capture);
 * nothing on the launch path reads the environment.  Defaults are the production kernels; at
 * sfa_model_create the env variable named beside each key seeds it, sfa_model_set_option
 * overrides it.  Not concurrently with a forward of this model.  (Round 4: the round-2/3 tune
 * bits, stem ablations, grouped heads and second side stream — measured and not adopted — moved to
 * tools/experiments/r03 with their convbench hooks.)
 *   SFA_OPT_STEM_PATCH  (SFA_STEM_PATCH)  1 (default): the fp16x3 stem + max-pool in one kernel
 *                                         over 16 x 16 patches + a merge pass; 0: the
 *                                         implicit-GEMM stem + the max-pool kernel
 *   SFA_OPT_FPN_COMMUTE (SFA_FPN_COMMUTE) bit mask of the FPN levels run commuted (7, fp16x3)
 *   SFA_OPT_FPN_GEMM    (SFA_FPN_GEMM)    bit mask of the commuted FPN 1x1 convs on the persistent
 *                                         weight-resident kernel: bit f = level f's low-resolution
 *                                         conv, bit 3 + f = its skip conv (61: the low-res convs of
 *                                         levels 0 and 2, the level-2 skip conv on full rows, the
 *                                         level-0 / 1 skip convs on flat pixel steps); the others on
 *                                         the per-tile kernels
 *   SFA_OPT_SPLITK_TICKETS (SFA_SPLITK_TICKETS) 1 (default): the split-K layer4 strip convs combine
 *                                         their slices in the conv kernel (the last slice of a tile to
 *                                         finish, by an atomic ticket); 0: a reduce launch per conv; the
 *                                         same bits
 */
enum sfa_model_option { SFA_OPT_STEM_PATCH = 0, SFA_OPT_FPN_COMMUTE = 1, SFA_OPT_FPN_GEMM = 2,
                        SFA_OPT_SPLITK_TICKETS = 3 };
int sfa_model_set_option(sfa_model* model, int key, int value);
int sfa_model_get_option(const sfa_model* model, int key, int* value);

/* Kernel probe (measurement only; no reference counterpart).  SFA_PROBE_HEADS: every
 * forward NOT being captured into a graph records a timing event before and after each
 * detection-head level's launch (the dominant kernel, 54.6 % of the FLOPs), on the stream
 * that launches it; SFA_PROBE_SERIAL: all launches stay on the caller's stream (no
 * side streams), so each head launch has the chip to itself.  sfa_model_probe_times
 * waits for the last probed forward's events and returns the launch durations of head
 * levels 0 .. n-1 in ms.  flags = 0 turns the probe off. */
enum sfa_probe_flags { SFA_PROBE_HEADS = 1, SFA_PROBE_SERIAL = 2 };
int sfa_model_set_probe(sfa_model* model, int flags);
int sfa_model_probe_times(const sfa_model* model, float* ms, int n);

/* Forward.  x: device float32, layout SFA_IN_NCHW3 (B,3,H,W) as the reference
 * takes it, SFA_IN_NHWC4 (B,H,W,4) as sfa_bev_voxelize writes it, or
 * SFA_IN_NCHW3_FLIP_HW: (B,3,H,W) read as torch.flip(x, [2, 3]) — the back view of
 * utils/demo_utils.py:110-111 do_detect, fused into the layout conversion.
 * H, W multiples of 32.  head_out[i]: device float32 (B, c_i, H/4, W/4) NCHW,
 * contiguous, forward head order — raw logits like the reference (no sigmoid).
 * workspace: sfa_forward_workspace_size(B, H, W) bytes.
 * Batch limit: the conv kernels address each input map with 32-bit byte offsets, so one pass
 * holds at most sfa_forward_max_batch(H, W) frames = floor((2^31 - 1) / (32 H W)) (the widest
 * conv input, up_level3, is 32 H W bytes per frame): 181 frames at 608 x 608.  A larger batch
 * runs as consecutive passes of that many frames on the caller's stream, sharing one workspace
 * sized for a pass (bit-identical per frame: the arithmetic is batch-invariant); a single frame
 * too large for one pass (H W >= 2^26) is refused with SFA_E_UNSUPPORTED before any launch. */
enum sfa_input_layout { SFA_IN_NCHW3 = 0, SFA_IN_NHWC4 = 1, SFA_IN_NCHW3_FLIP_HW = 2 };
int sfa_forward_max_batch(int height, int width);
size_t sfa_forward_workspace_size(const sfa_model* model, int batch, int height, int width);
int sfa_model_forward(const sfa_model* model, const float* x, int in_layout, int batch, int height,
                      int width, float* const* head_out, void* workspace, size_t workspace_bytes,
                      void* stream);

/* Byte offset inside the forward workspace of an intermediate map, valid after
 * sfa_model_forward returns on the stream (for the reference's opt-in
 * visualisation capture, fpn_resnet.py:189-242).  LAYERk / UP_LEVELk are NHWC
 * float32 (B, h, w, C); HEADS_Lk are channel-planar float32
 * [sum(head_channels)][B][h][w] per KFPN level.  -1 on bad arguments. */
enum sfa_buffer {
  SFA_BUF_LAYER1 = 0, SFA_BUF_LAYER2, SFA_BUF_LAYER3, SFA_BUF_LAYER4,
  SFA_BUF_UP_LEVEL2, SFA_BUF_UP_LEVEL3, SFA_BUF_UP_LEVEL4,
  SFA_BUF_HEADS_L0, SFA_BUF_HEADS_L1, SFA_BUF_HEADS_L2
};
int64_t sfa_forward_buffer_offset(const sfa_model* model, int batch, int height, int width,
                                  int which);

/* --------------------------------------------------------------- decode --
 * Replaces utils/torch_utils.py:44-45 _sigmoid (in place: sigmoid then
 * clamp(1e-4, 1-1e-4)). */
int sfa_sigmoid_clamp_inplace(float* x, int64_t n, void* stream);

/* Replaces utils/evaluation_utils.py:77-105 decode (with _nms :21-26, _topk
 * :47-62, _transpose_and_gather_feat :40-44).  All maps device float32 NCHW
 * contiguous: hm (B,C,H,W), off (B,2,H,W) or NULL, dir (B,2,H,W),
 * z (B,1,H,W), dim (B,3,H,W).  apply_sigmoid != 0 applies _sigmoid to hm and
 * off on the fly (the test.py:150,167 pair) without modifying them.
 * dets: device float32 (B, K, 10) columns
 *   [score, xs+off0, ys+off1, z, dim0, dim1, dim2, dir0, dir1, class].
 * Ties (unspecified order in torch.topk) break by lower flat index, then lower
 * class.  Constraints: K <= 256, K <= H*W, H*W <= 36864, C <= 16.
 * workspace: sfa_decode_workspace_size(B, C, K) bytes. */
size_t sfa_decode_workspace_size(int batch, int num_classes, int K);
int sfa_decode(const float* hm, const float* off, const float* dir, const float* z,
               const float* dim, int batch, int num_classes, int height, int width, int K,
               int apply_sigmoid, float* dets, void* workspace, size_t workspace_bytes,
               void* stream);

/* The reference's decode helpers, each on its own (utils/evaluation_utils.py; the drop-in
 * utils.evaluation_utils serves them from these, so no caller falls through to torch code):
 *
 * sfa_heat_nms replaces :21-26 _nms(heat, kernel=3): out = heat * (max_pool2d(heat, 3, 1, 1) ==
 * heat) over `maps` float32 maps of height x width (pool padded with -inf; non-peaks become the
 * signed zero of the multiply).  out must not alias heat.
 *
 * sfa_topk replaces :47-62 _topk(scores, K) (per_channel = 0) and :65-74 _topk_channel
 * (per_channel = 1) on float32 (B, C, H, W) scores (no peak test; decode's sfa_decode fuses it):
 *   per_channel = 0: out_scores f32 (B, K), out_inds int64 (B, K) (flat index within the class
 *     map), out_clses int32 (B, K), out_ys / out_xs f32 (B, K) = floor(ind / W), ind % W;
 *   per_channel = 1: out_scores, out_inds, out_ys, out_xs of shape (B, C, K); out_clses unused.
 * Each class's K by (value desc, index asc), then the classes' C*K by (value desc, class asc,
 * rank asc) — torch.topk's two stages, its unspecified tie order made definite.  Constraints as
 * sfa_decode (K <= 256, K <= H*W <= 36864, C <= 16); workspace sfa_topk_workspace_size(B, C, K).
 *
 * sfa_gather_feat replaces :29-37 _gather_feat(feat, ind) (mask None: stride_n = dim, stride_d = 1,
 * feat (B, n, dim)) and :40-44 _transpose_and_gather_feat (feat (B, dim, H, W): n = H*W,
 * stride_n = 1, stride_d = H*W): out[b][k][d] = feat[b*n*dim + ind[b][k]*stride_n + d*stride_d],
 * elements of elem_bytes 4 (f32 / int32) or 8 (int64); ind int64 (B, K) in [0, n), checked by the
 * caller (torch.gather's contract). */
int sfa_heat_nms(const float* heat, float* out, int64_t maps, int height, int width, void* stream);
size_t sfa_topk_workspace_size(int batch, int num_classes, int K);
int sfa_topk(const float* scores, int batch, int num_classes, int height, int width, int K, int per_channel,
             float* out_scores, int64_t* out_inds, int32_t* out_clses, float* out_ys, float* out_xs,
             void* workspace, size_t workspace_bytes, void* stream);
int sfa_gather_feat(const void* feat, int batch, int64_t n, int dim, int64_t stride_n, int64_t stride_d,
                    int elem_bytes, const int64_t* ind, int K, void* out, void* stream);

/* ------------------------------------------------ post-processing on device --
 * the SFA side of the fusion scripts without a host hop.
 *
 * sfa_post_process replaces utils/evaluation_utils.py:112-163 post_processing (for
 * EVERY frame; the reference returns only the last one, :158) followed by :177-193
 * convert_det_to_real_values.  dets: device f32 (B, K, 10) from sfa_decode.  Per frame
 * the rows with class == j and score > peak_thresh (f32 compare), class-major, decode
 * order within a class, are written compacted (frame b at out_offsets[b], a DEVICE
 * int32 array of batch+1 entries written by the call):
 *   out_preds f32 (n, 8) [score, x*down, y*down, z, h, w/bound_y*bev_w, l/bound_x*bev_h,
 *                         atan2(dir0, dir1)]          (the post_processing dict rows)
 *   out_real  f64 (n, 8) [class, x, y, z, h, w, l, yaw] (convert_det_to_real_values)
 * convert_det_to_real_values works on numpy scalars, so its arithmetic type follows the
 * numpy version: SFA_REAL_F32 = numpy >= 2 (f32, as the fixtures were generated),
 * SFA_REAL_F64 = numpy 1.x (f64 from the f32 inputs; requirements.txt pins 1.18.3).
 * Capacity: batch*K rows.  One workgroup (the work is a few hundred rows). */
enum sfa_real_arith { SFA_REAL_F32 = 0, SFA_REAL_F64 = 1 };
typedef struct sfa_post_params {
  int num_classes;        /* 3 */
  int down_ratio;         /* 4 */
  float peak_thresh;      /* 0.2 */
  int bev_h, bev_w;       /* 608, 608 (kitti_config.py BEV_HEIGHT / BEV_WIDTH) */
  double bound_x, bound_y;            /* 50, 50 */
  double min_x, min_y, min_z;         /* 0, -25, -2.73 */
  int arith;              /* SFA_REAL_F32 | SFA_REAL_F64 */
} sfa_post_params;
int sfa_post_process(const float* dets, int batch, int K, const sfa_post_params* params,
                     float* out_preds, double* out_real, int32_t* out_offsets, void* stream);

/* sfa_project_boxes replaces test6.py:129-187 convert_sfa3d_to_2d_boxes (with
 * data_process/transformation.py:99-107 lidar_to_camera_box): for each real row
 * (CSR by DEVICE offsets) whose confidence >= conf_min — the confidence is column 0
 * (the class id, as the reference reads it, test6.py:138) with SFA_CONF_CLASS_ID or the
 * detection score (preds column 0) with SFA_CONF_SCORE — the 8 box corners are moved
 * to the camera (V2C, R0), rotated by ry = -yaw - pi/2, projected with P2, clipped to
 * the image like Python max(0, .) / min(img, .), and kept when max > min as int32
 * [int(min_x), int(min_y), int(max_x - min_x), int(max_y - min_y)].
 * Outputs compacted per frame (out_offsets, DEVICE int32 batch+1, written by the
 * call): boxes int32 (m, 4), conf f64, out_row = the row index within the frame's
 * real rows, out_extent (optional) f64 (m, 4) = clipped [min_x, min_y, max_x, max_y].
 * calib: DEVICE array of `batch` sfa_calib (or one, when calib_per_frame = 0); the
 * matrices are the calib file's values (f32 in the reference, widened to f64).
 * f64 without contraction; numpy's BLAS and libm may differ in the last ulp. */
enum sfa_conf_source { SFA_CONF_CLASS_ID = 0, SFA_CONF_SCORE = 1 };
typedef struct sfa_calib {
  double V2C[12];  /* Tr_velo_to_cam 3x4, row-major */
  double R0[9];    /* R_rect 3x3 */
  double P2[12];   /* 3x4 */
  int32_t img_h, img_w;
} sfa_calib;
typedef struct sfa_project_params {
  double conf_min;      /* 0.3 */
  int conf_source;      /* SFA_CONF_CLASS_ID | SFA_CONF_SCORE */
  int calib_per_frame;  /* 1: calib[b] per frame; 0: calib[0] for all */
} sfa_project_params;
int sfa_project_boxes(const double* real, const float* preds, const int32_t* offsets, int batch,
                      const sfa_calib* calib, const sfa_project_params* params,
                      int32_t* out_boxes, double* out_conf, int32_t* out_row, double* out_extent,
                      int32_t* out_offsets, void* stream);

/* ------------------------------------------------------- .bin streaming --
 * KITTI velodyne .bin files (data_process/kitti_dataset.py:119-122
 * get_lidar = np.fromfile(path, float32).reshape(-1, 4)) read in batches by a producer
 * thread with n_threads pread() workers into two host staging slots, overlapped with
 * the GPU work of the previous batch.  pinned = 1: slots are hipHostMalloc'd and
 * sfa_bin_stream_next copies a batch to DEVICE `points` with hipMemcpyAsync on
 * `stream` (the slot is reused only after that copy completed); pinned = 0: plain host
 * slots, `points` is a HOST buffer (memcpy; no device involved).  The stream allocates
 * its own host memory (2 x max_points_per_batch x 16 B), never device memory.
 * next() fills frame_offsets (HOST, batch + 1 entries, ready for sfa_bev_voxelize) and
 * *n_frames (< batch for the last partial batch, 0 at the end).  A file whose float
 * count is not a multiple of 4 fails the batch (the reference's reshape raises). */
typedef struct sfa_bin_stream sfa_bin_stream;
int sfa_bin_stream_create(const char* const* paths, int n_files, int batch,
                          int64_t max_points_per_batch, int n_threads, int pinned,
                          sfa_bin_stream** out);
int sfa_bin_stream_next(sfa_bin_stream* s, float* points, int64_t capacity_points,
                        int64_t* frame_offsets, int* n_frames, void* stream);
void sfa_bin_stream_destroy(sfa_bin_stream* s);

/* ------------------------------------------------------------ fusion --
 * Camera-LiDAR late fusion + NMS.  Replaces test6.py:310-348
 * create_fused_detections_wrapper -> :231-308 bayesian_inspired_fuse_overlapping_detections
 * (mode SFA_FUSE_BAYES) or test5.py:285-321 create_fused_detections -> :213-282
 * fuse_overlapping_detections (SFA_FUSE_WEIGHTED), then test6.py:104-126
 * apply_nms_to_fused_detections, all with test6.py:76-101 calculate_iou.
 *
 * Per frame b (CSR by DEVICE int32 offsets [batch+1]): YOLO boxes int32 [x,y,w,h],
 * f64 confidence, int32 class id; SFA 2D boxes int32 [x,y,w,h], f64 confidence.
 * At most 512 boxes per side per frame (a larger frame gets out_count = -1).
 * Output for frame b starts at element yolo_offsets[b] + sfa_offsets[b] (capacity
 * = its yolo + sfa count): the fused list in the reference's order (fused/kept YOLO
 * entries in YOLO order, then unmatched SFA), source SFA_SRC_*, class id (SFA: 0);
 * out_origin (optional) = index of the entry in its frame's INPUT list (YOLO for
 * YOLO/fused entries, SFA for SFA entries), out_match (optional) = the SFA input
 * index fused into a fused entry, else -1;
 * out_keep = indices into that list of the NMS survivors, in NMS output order.
 * All f64 arithmetic is IEEE without contraction: bit-identical to the Python. */
enum sfa_fuse_mode { SFA_FUSE_BAYES = 0, SFA_FUSE_WEIGHTED = 1 };
enum sfa_fuse_source { SFA_SRC_YOLO = 0, SFA_SRC_LIDAR = 1, SFA_FUSED = 2 };
typedef struct sfa_fusion_params {
  double conf_threshold;        /* keep detections with conf >= this (default 0.3) */
  double fusion_iou_threshold;  /* associate when IoU >= this (default 0.7) */
  double nms_threshold;         /* suppress when IoU > this (default 0.5) */
  int mode;                     /* SFA_FUSE_BAYES | SFA_FUSE_WEIGHTED */
  int apply_nms;                /* 0: fusion only */
} sfa_fusion_params;

/* IoU matrix out[i][j] = calculate_iou(a[i], b[j]) (test6.py:76-101), f64. */
int sfa_iou_matrix(const int32_t* boxes_a, int na, const int32_t* boxes_b, int nb, double* out,
                   void* stream);

/* Gaussian soft-NMS: replaces README.md:250-261 gaussian_nms(detections, sigma=0.5) (the
 * reference's only definition of it): for each frame b, the count[b] detections at
 * boxes/conf[start[b] ..] (DEVICE int32 starts/counts [batch]; boxes int32 [x,y,w,h] as
 * calculate_iou, test6.py:76-101) are visited in order and every later one decays in place,
 * conf[j] *= exp(-iou(i, j)^2 / sigma) for i < j in increasing i; order, boxes and count are
 * unchanged (no threshold).  f64; a count <= 0 leaves the frame untouched.  Chains after
 * sfa_fuse_detections with starts = yolo_offsets[b] + sfa_offsets[b], counts = out_count. */
int sfa_gaussian_nms(int batch, const int32_t* boxes, double* conf, const int32_t* starts,
                     const int32_t* counts, double sigma, void* stream);

int sfa_fuse_detections(int batch, const int32_t* yolo_boxes, const double* yolo_conf,
                        const int32_t* yolo_cls, const int32_t* yolo_offsets,
                        const int32_t* sfa_boxes, const double* sfa_conf,
                        const int32_t* sfa_offsets, const sfa_fusion_params* params,
                        int32_t* out_boxes, double* out_conf, int32_t* out_cls, int32_t* out_src,
                        int32_t* out_origin, int32_t* out_match, int32_t* out_count,
                        int32_t* out_keep, int32_t* out_keep_count, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SFA_HIP_H_ */
