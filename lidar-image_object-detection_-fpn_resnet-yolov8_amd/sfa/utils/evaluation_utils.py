"""Drop-in for the reference's utils/evaluation_utils.py.

* ``decode`` (:77-105, with _nms :21-26, _topk :47-62, gathers :29-44) runs as
  two HIP kernels (sfa_decode) on the input's GPU and returns (B, K, 10) float32
  on that device.  Equal scores, whose order torch.topk leaves unspecified, are
  ordered by lower flat index, then lower class.
* ``post_processing`` (:112-163) is the reference's HOST function on the numpy
  detections the caller already copied back (test.py:172); it keeps the
  reference's quirk of returning only the LAST frame's dict (``ret.append`` sits
  outside the frame loop, :158).  ``post_processing_batch`` returns every frame.
  The reference's per-array prints are emitted only when SFA_VERBOSE=1.
* ``convert_det_to_real_values`` (:177-193), ``get_yaw`` (:108-109) and
  ``draw_predictions`` (:166-174, needs OpenCV) are host-side like the reference.
* The decode helpers, for callers that use them on their own: ``_nms`` (:21-26,
  sfa_heat_nms), ``_topk`` (:47-62) and ``_topk_channel`` (:65-74, sfa_topk),
  ``_gather_feat`` (:29-37) and ``_transpose_and_gather_feat`` (:40-44, sfa_gather_feat) run on
  the GPU too (no name of the hot path falls through to the reference's torch code); ties in
  the top-K ordered as in ``decode``.  ``_gather_feat`` with a ``mask`` (its boolean selection
  has a data-dependent shape; the reference never passes one) raises NotImplementedError.
"""

from __future__ import annotations

import os

import numpy as np

import config.kitti_config as cnf
from sfa_hip import runtime
from sfa_hip import dropin as _dropin

_VERBOSE = os.environ.get("SFA_VERBOSE", "0") == "1"


def _nms(heat, kernel=3):
    if kernel != 3:
        raise NotImplementedError(f"_nms: the HIP kernel implements kernel = 3 (got {kernel})")
    return runtime.heat_nms(heat)


def _gather_feat(feat, ind, mask=None):
    if mask is not None:
        raise NotImplementedError("_gather_feat with a mask (data-dependent shape) is not on the gfx950 path")
    return runtime.gather_feat(feat, ind)


def _transpose_and_gather_feat(feat, ind):
    return runtime.gather_feat(feat, ind, transpose=True)


def _topk(scores, K=40):
    return runtime.topk(scores, K)


def _topk_channel(scores, K=40):
    return runtime.topk(scores, K, per_channel=True)


def decode(hm_cen, cen_offset, direction, z_coor, dim, K=40):
    return runtime.decode(hm_cen, cen_offset, direction, z_coor, dim, K=K, apply_sigmoid=False)


def get_yaw(direction):
    return np.arctan2(direction[:, 0:1], direction[:, 1:2])


def _frame_preds(det, num_classes, down_ratio, peak_thresh, i):
    top_preds = {}
    classes = det[:, -1]
    if _VERBOSE:
        print(f"Processing batch {i}, number of detections: {len(classes)}")
    for j in range(num_classes):
        sel = det[classes == j]
        # x, y, z, h, w, l, yaw in BEV pixels (:136-144)
        preds = np.concatenate([
            sel[:, 0:1],
            sel[:, 1:2] * down_ratio,
            sel[:, 2:3] * down_ratio,
            sel[:, 3:4],
            sel[:, 4:5],
            sel[:, 5:6] / cnf.bound_size_y * cnf.BEV_WIDTH,
            sel[:, 6:7] / cnf.bound_size_x * cnf.BEV_HEIGHT,
            get_yaw(sel[:, 7:9]).astype(np.float32)], axis=1)
        if len(preds) > 0:
            preds = preds[preds[:, 0] > peak_thresh]
        if _VERBOSE:
            print(f"Class {j} has {len(preds)} detections after peak_thresh={peak_thresh}.")
        top_preds[j] = preds
    return top_preds


def post_processing(detections, num_classes=3, down_ratio=4, peak_thresh=0.2):
    """Reference semantics: a list holding ONE dict — the last frame's (:158)."""
    if _VERBOSE:
        print(f"Input detections shape: {detections.shape}")
    if detections.shape[0] == 0:
        return []
    last = detections.shape[0] - 1
    return [_frame_preds(detections[last], num_classes, down_ratio, peak_thresh, last)]


def post_processing_batch(detections, num_classes=3, down_ratio=4, peak_thresh=0.2):
    """Every frame's dict (what the reference loop evidently intended)."""
    return [_frame_preds(detections[i], num_classes, down_ratio, peak_thresh, i)
            for i in range(detections.shape[0])]


def draw_predictions(img, detections, num_classes=3):
    from data_process.kitti_bev_utils import drawRotatedBox
    for j in range(num_classes):
        for det in detections[j]:
            _score, _x, _y, _z, _h, _w, _l, _yaw = det
            drawRotatedBox(img, _x, _y, _w, _l, _yaw, cnf.colors[int(j)])
    return img


def convert_det_to_real_values(detections, num_classes=3):
    kitti_dets = []
    for cls_id in range(num_classes):
        for det in detections[cls_id]:
            _score, _x, _y, _z, _h, _w, _l, _yaw = det
            kitti_dets.append([
                cls_id,
                _y / cnf.BEV_HEIGHT * cnf.bound_size_x + cnf.boundary["minX"],
                _x / cnf.BEV_WIDTH * cnf.bound_size_y + cnf.boundary["minY"],
                _z + cnf.boundary["minZ"],
                _h,
                _w / cnf.BEV_WIDTH * cnf.bound_size_y,
                _l / cnf.BEV_HEIGHT * cnf.bound_size_x,
                -_yaw])
    return np.array(kitti_dets)


# names of the reference module this drop-in does not define come from the reference
__getattr__ = _dropin.module_getattr(__name__)
