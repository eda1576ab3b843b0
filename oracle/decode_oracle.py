"""Decode / post-processing oracle (numpy) — TEST INFRASTRUCTURE ONLY.

Restates utils/torch_utils.py:44-45 and utils/evaluation_utils.py:21-193:

* ``sigmoid_clamp``   torch_utils.py:44-45: sigmoid then clamp(1e-4, 1-1e-4), f32.
* ``nms_peaks``       evaluation_utils.py:21-26: 3x3/s1 max-pool with -inf padding;
                      keep = (hmax == heat); heat * keep (plateaus all survive).
* ``topk``            evaluation_utils.py:47-62: per-class top-K over H*W, then
                      top-K over the (C*K) survivors; class = idx // K.  torch leaves
                      the order of equal scores unspecified (SURVEY §7 hard part 2);
                      this oracle — and the HIP kernel — break ties by the lower
                      flat index (stage 1) and the lower (class*K + rank) (stage 2).
* ``decode``          evaluation_utils.py:77-105: gather offset/direction/z/dim at the
                      peak; columns [score, xs+off0, ys+off1, z, dim0..2, dir0, dir1, cls].
* ``post_processing`` evaluation_utils.py:112-163 (prints dropped); the reference
                      returns only the LAST frame's dict (``ret.append`` is outside
                      the frame loop, :158) — reproduced; ``post_processing_all``
                      returns every frame.
* ``convert_det_to_real_values`` evaluation_utils.py:177-193.
"""

from __future__ import annotations

import numpy as np

BEV_W = 608
BEV_H = 608
BOUND_X = 50.0
BOUND_Y = 50.0
MIN_X, MIN_Y, MIN_Z = 0.0, -25.0, -2.73


def sigmoid_clamp(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32)
    s = (np.float32(1.0) / (np.float32(1.0) + np.exp(-x))).astype(np.float32)
    return np.clip(s, np.float32(1e-4), np.float32(1 - 1e-4)).astype(np.float32)


def nms_peaks(heat: np.ndarray) -> np.ndarray:
    """heat (B, C, H, W) f32 -> heat where it equals its 3x3 neighbourhood max, else 0."""
    B, C, H, W = heat.shape
    p = np.full((B, C, H + 2, W + 2), -np.inf, dtype=np.float32)
    p[:, :, 1:-1, 1:-1] = heat
    hmax = np.full_like(heat, -np.inf)
    for dy in range(3):
        for dx in range(3):
            hmax = np.maximum(hmax, p[:, :, dy:dy + H, dx:dx + W])
    return (heat * (hmax == heat)).astype(np.float32)


def _topk_desc(vals: np.ndarray, k: int):
    """Top-k of a 1-D array: descending value, ties by lower index."""
    order = np.lexsort((np.arange(vals.size), -vals.astype(np.float64)))
    sel = order[:k]
    return vals[sel], sel


def topk(scores: np.ndarray, K: int):
    B, C, H, W = scores.shape
    flat = scores.reshape(B, C, H * W)
    s1 = np.zeros((B, C, K), np.float32)
    i1 = np.zeros((B, C, K), np.int64)
    for b in range(B):
        for c in range(C):
            s1[b, c], i1[b, c] = _topk_desc(flat[b, c], K)
    ys1 = (i1 // W).astype(np.float32)
    xs1 = (i1 % W).astype(np.float32)
    score = np.zeros((B, K), np.float32)
    ind = np.zeros((B, K), np.int64)
    cls = np.zeros((B, K), np.int32)
    ys = np.zeros((B, K), np.float32)
    xs = np.zeros((B, K), np.float32)
    for b in range(B):
        sc, j = _topk_desc(s1[b].reshape(-1), K)
        score[b] = sc
        cls[b] = (j // K).astype(np.int32)
        ind[b] = i1[b].reshape(-1)[j]
        ys[b] = ys1[b].reshape(-1)[j]
        xs[b] = xs1[b].reshape(-1)[j]
    return score, ind, cls, ys, xs


def _gather(feat: np.ndarray, ind: np.ndarray) -> np.ndarray:
    """feat (B, C, H, W), ind (B, K) -> (B, K, C)  (_transpose_and_gather_feat)."""
    B, C, H, W = feat.shape
    f = feat.reshape(B, C, H * W)
    return np.stack([f[b][:, ind[b]].T for b in range(B)]).astype(np.float32)


def decode(hm_cen, cen_offset, direction, z_coor, dim, K=40):
    B = hm_cen.shape[0]
    heat = nms_peaks(hm_cen)
    score, ind, cls, ys, xs = topk(heat, K)
    if cen_offset is not None:
        off = _gather(cen_offset, ind)
        xs = xs[:, :, None] + off[:, :, 0:1]
        ys = ys[:, :, None] + off[:, :, 1:2]
    else:
        xs = xs[:, :, None] + np.float32(0.5)
        ys = ys[:, :, None] + np.float32(0.5)
    dirn = _gather(direction, ind)
    z = _gather(z_coor, ind)
    d = _gather(dim, ind)
    return np.concatenate([score.reshape(B, K, 1), xs, ys, z, d, dirn,
                           cls.reshape(B, K, 1).astype(np.float32)], axis=2).astype(np.float32)


def _frame_post(det: np.ndarray, num_classes, down_ratio, peak_thresh) -> dict:
    out = {}
    classes = det[:, -1]
    for j in range(num_classes):
        sel = det[classes == j]
        rows = np.concatenate([
            sel[:, 0:1], sel[:, 1:2] * down_ratio, sel[:, 2:3] * down_ratio, sel[:, 3:4], sel[:, 4:5],
            sel[:, 5:6] / BOUND_Y * BEV_W, sel[:, 6:7] / BOUND_X * BEV_H,
            np.arctan2(sel[:, 7:8], sel[:, 8:9]).astype(np.float32)], axis=1)
        if len(rows) > 0:
            rows = rows[rows[:, 0] > peak_thresh]
        out[j] = rows
    return out


def post_processing(detections, num_classes=3, down_ratio=4, peak_thresh=0.2):
    if detections.shape[0] == 0:
        return []
    return [_frame_post(detections[-1], num_classes, down_ratio, peak_thresh)]


def post_processing_all(detections, num_classes=3, down_ratio=4, peak_thresh=0.2):
    return [_frame_post(d, num_classes, down_ratio, peak_thresh) for d in detections]


def convert_det_to_real_values(detections, num_classes=3):
    rows = []
    for cls_id in range(num_classes):
        for det in detections[cls_id]:
            _s, _x, _y, _z, _h, _w, _l, _yaw = det
            rows.append([cls_id, _y / BEV_H * BOUND_X + MIN_X, _x / BEV_W * BOUND_Y + MIN_Y,
                         _z + MIN_Z, _h, _w / BEV_W * BOUND_Y, _l / BEV_H * BOUND_X, -_yaw])
    return np.array(rows)
