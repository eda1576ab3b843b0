"""Detections -> metres -> camera image boxes oracle (numpy) — TEST INFRASTRUCTURE ONLY.

Restates, per frame, the SFA side of the fusion scripts:

* ``post_frame``      evaluation_utils.py:112-163 for ONE frame (decode_oracle._frame_post):
                      class-major rows [score, x*4, y*4, z, h, w/50*608, l/50*608,
                      atan2(im, re)] in f32, kept when score > peak_thresh (f32 compare).
* ``real_rows``       evaluation_utils.py:177-193 convert_det_to_real_values.  The
                      reference does this on numpy *scalars* (``for det in ...``), so the
                      arithmetic type depends on the numpy version: numpy >= 2 (NEP 50,
                      the container that generated the fixtures) keeps f32; numpy 1.x
                      (requirements.txt pins 1.18.3) promotes f32-scalar ⊕ Python number
                      to f64.  ``arith="f32"`` is fixture-pinned; ``arith="f64"`` restates
                      the numpy 1.x rules (parity unpinned: numpy 1.x is not installed).
* ``lidar_to_camera`` transformation.py:50-59 / :99-107 lidar_to_camera_box with a
                      calibration: V2C @ [x,y,z,1], then R0 @ ·; ry = -rz - pi/2.
* ``image_boxes``     test6.py:129-187 convert_sfa3d_to_2d_boxes: skip rows whose column
                      0 (the CLASS ID — the reference's quirk) is < 0.3, 8 corners rotated
                      about y, P2 projection, min/max, clip with Python max(0, ·) /
                      min(img, ·), keep when max > min, int() truncation; the "confidence"
                      returned is that class id.

BLAS (numpy matmul / dot) and the SIMD arctan2 make the f64 corner values and the f32
yaw platform dependent at the last ulp: tests compare those within a stated tolerance
and the int boxes exactly.
"""

from __future__ import annotations

import math

import numpy as np

from . import decode_oracle as do

BEV_W = BEV_H = 608
BOUND_X = BOUND_Y = 50
MIN_X, MIN_Y, MIN_Z = 0, -25, -2.73


def post_frame(det, num_classes=3, down_ratio=4, peak_thresh=0.2):
    """evaluation_utils.py:129-157 for one frame -> {cls: (n, 8) f32}."""
    return do._frame_post(det, num_classes, down_ratio, peak_thresh)


def real_rows(preds, num_classes=3, arith="f32"):
    """evaluation_utils.py:177-193 -> (n, 8) f64 [cls, x, y, z, h, w, l, yaw]."""
    rows = []
    for cls_id in range(num_classes):
        for det in preds[cls_id]:
            _s, _x, _y, _z, _h, _w, _l, _yaw = (np.float32(v) for v in det)
            if arith == "f32":  # numpy >= 2: f32 scalar with Python int/float stays f32
                f = np.float32
                x = _y / f(BEV_H) * f(BOUND_X) + f(MIN_X)
                y = _x / f(BEV_W) * f(BOUND_Y) + f(MIN_Y)
                z = _z + f(MIN_Z)
                w = _w / f(BEV_W) * f(BOUND_Y)
                l = _l / f(BEV_H) * f(BOUND_X)
            else:  # numpy 1.x: promoted to f64
                x = float(_y) / BEV_H * BOUND_X + MIN_X
                y = float(_x) / BEV_W * BOUND_Y + MIN_Y
                z = float(_z) + MIN_Z
                w = float(_w) / BEV_W * BOUND_Y
                l = float(_l) / BEV_H * BOUND_X
            rows.append([cls_id, x, y, z, _h, w, l, -_yaw])
    return np.array(rows, dtype=np.float64).reshape(-1, 8)


def lidar_to_camera(box, V2C, R0):
    """transformation.py:50-59,99-107 for one (7,) box -> (7,) camera box."""
    x, y, z, h, w, l, rz = (float(v) for v in box)
    V2C = np.asarray(V2C, np.float64).reshape(3, 4)
    R0 = np.asarray(R0, np.float64).reshape(3, 3)
    p = [x, y, z, 1.0]
    c = [sum_lr(V2C[i, k] * p[k] for k in range(4)) for i in range(3)]
    r = [sum_lr(R0[i, k] * c[k] for k in range(3)) for i in range(3)]
    return np.array([r[0], r[1], r[2], h, w, l, -rz - np.pi / 2])


def sum_lr(terms):
    s = 0.0
    first = True
    for t in terms:
        s = t if first else s + t
        first = False
    return s


def box_corners_2d(cam_box, P2):
    """test6.py:148-171: 8 corners -> image (u, v) arrays (f64)."""
    x, y, z, h, w, l, ry = (float(v) for v in cam_box)
    P2 = np.asarray(P2, np.float64).reshape(3, 4)
    cx = [-l / 2, -l / 2, l / 2, l / 2, -l / 2, -l / 2, l / 2, l / 2]
    cy = [0.0, 0.0, 0.0, 0.0, -h, -h, -h, -h]
    cz = [-w / 2, w / 2, w / 2, -w / 2, -w / 2, w / 2, w / 2, -w / 2]
    c, s = math.cos(ry), math.sin(ry)
    u, v = [], []
    for k in range(8):
        X = c * cx[k] + s * cz[k] + x
        Y = cy[k] + y
        Z = -s * cx[k] + c * cz[k] + z
        q = [X, Y, Z, 1.0]
        pu = sum_lr(P2[0, m] * q[m] for m in range(4))
        pv = sum_lr(P2[1, m] * q[m] for m in range(4))
        pw = sum_lr(P2[2, m] * q[m] for m in range(4))
        u.append(pu / pw)
        v.append(pv / pw)
    return np.array(u), np.array(v)


def _py_max0(v):  # Python max(0, v): v only when v > 0
    return v if v > 0 else 0.0


def _py_minimg(lim, v):  # Python min(lim, v): v only when v < lim
    return v if v < lim else float(lim)


def image_boxes(real, calib, img_shape, conf_min=0.3, conf=None):
    """test6.py:129-187 on (n, 8) real rows -> (boxes int (m,4), conf f64 (m,), rows (m,),
    extents f64 (m, 4) = the clipped [min_x, min_y, max_x, max_y] before int()).
    ``conf`` defaults to column 0 (the class id, as the reference reads it); pass the
    detection scores for the score-confidence variant."""
    boxes, conf_out, rows, ext = [], [], [], []
    for i, det in enumerate(real):
        cf = det[0] if conf is None else conf[i]
        if cf < conf_min:
            continue
        cam = lidar_to_camera(det[1:], calib["V2C"], calib["R0"])
        u, v = box_corners_2d(cam, calib["P2"])
        mnx, mxx = np.min(u), np.max(u)
        mny, mxy = np.min(v), np.max(v)
        mnx, mny = _py_max0(mnx), _py_max0(mny)
        mxx, mxy = _py_minimg(img_shape[1], mxx), _py_minimg(img_shape[0], mxy)
        if mxx > mnx and mxy > mny:
            boxes.append([int(mnx), int(mny), int(mxx - mnx), int(mxy - mny)])
            conf_out.append(float(cf))
            rows.append(i)
            ext.append([mnx, mny, mxx, mxy])
    return (np.array(boxes, np.int64).reshape(-1, 4), np.array(conf_out, np.float64),
            np.array(rows, np.int64), np.array(ext, np.float64).reshape(-1, 4))


def run_frames(dets, calibs, img_shapes, arith="f32", peak_thresh=0.2, conf_min=0.3,
               score_conf=False):
    """All frames: dets (B, K, 10) f32 -> per-frame (preds dict, real, boxes tuple)."""
    out = []
    for b in range(dets.shape[0]):
        preds = post_frame(dets[b], 3, 4, peak_thresh)
        real = real_rows(preds, 3, arith)
        sc = np.concatenate([preds[j][:, 0] for j in range(3)]).astype(np.float64) if score_conf \
            else None
        out.append((preds, real, image_boxes(real, calibs[b], img_shapes[b], conf_min, sc)))
    return out
