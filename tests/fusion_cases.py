"""Seeded inputs for the fusion fixtures (shared by the generator and the tests).

Boxes are [x, y, w, h] ints (YOLO's int(xyxy) boxes, test6.py:200-206; SFA's
int-cast projected boxes, :182); YOLO confidences are Python floats of f32
values (float(box.conf[0])); SFA "confidences" are either the reference's class-id
values 0/1/2 (the test6.py:138 quirk: column 0 of convert_det_to_real_values is
cls_id) or continuous scores.
"""

import numpy as np

from sfa_hip import synthetic

CLASS_NAMES = [f"class{i}" for i in range(80)]
IMG_W, IMG_H = 1242, 375


def _boxes(seed, stream, n):
    u = synthetic.hash_uniform(seed, stream, 4 * n).reshape(n, 4)
    x = (u[:, 0] * (IMG_W - 40)).astype(np.int64)
    y = (u[:, 1] * (IMG_H - 40)).astype(np.int64)
    w = (10 + u[:, 2] * 190).astype(np.int64)
    h = (10 + u[:, 3] * 140).astype(np.int64)
    return np.stack([x, y, w, h], 1)


def _case(seed, ny, ns, n_overlap, quirk_conf, conf_thr=0.3, fusion_iou=0.7, nms_thr=0.5,
          jitter=4):
    yb = _boxes(seed, 1, ny)
    yc = synthetic.hash_uniform(seed, 2, ny).astype(np.float32).astype(np.float64)
    ycls = (synthetic.hash_uniform(seed, 3, ny) * 80).astype(np.int64)
    sb = _boxes(seed, 4, ns)
    k = min(n_overlap, ny, ns)
    if k:
        jit = np.rint((synthetic.hash_uniform(seed, 5, 4 * k).reshape(k, 4) - 0.5) * 2 * jitter)
        sb[:k] = np.maximum(yb[:k] + jit.astype(np.int64), [0, 0, 1, 1])
    if quirk_conf:
        sc = np.floor(synthetic.hash_uniform(seed, 6, ns) * 3).astype(np.float64)
    else:
        sc = synthetic.hash_uniform(seed, 6, ns)
    return dict(yolo_boxes=[list(map(int, b)) for b in yb], yolo_conf=[float(c) for c in yc],
                yolo_cls=[int(c) for c in ycls], sfa_boxes=[list(map(int, b)) for b in sb],
                sfa_conf=[float(c) for c in sc], conf_thr=conf_thr, fusion_iou=fusion_iou,
                nms_thr=nms_thr)


def cases():
    c = {
        "typical": _case(1, 20, 10, 8, False),
        "quirk_conf": _case(2, 24, 12, 10, True),
        "low_fusion_thr": _case(3, 40, 30, 25, False, fusion_iou=0.3, nms_thr=0.3, jitter=12),
        "many": _case(4, 120, 90, 70, False, fusion_iou=0.5, jitter=8),
        "no_sfa": _case(5, 15, 0, 0, False),
        "no_yolo": _case(6, 0, 12, 0, False),
        "empty": _case(7, 0, 0, 0, False),
        "all_filtered": _case(8, 10, 10, 5, False, conf_thr=1.5),
    }
    # exact duplicates and ties: equal IoU candidates (first SFA index must win),
    # equal confidences (stable NMS order), zero-area boxes (union 0 -> IoU 0)
    d = _case(9, 6, 6, 0, False, fusion_iou=0.5)
    d["yolo_boxes"] = [[100, 100, 50, 40], [100, 100, 50, 40], [300, 50, 0, 30],
                       [500, 200, 60, 60], [700, 100, 30, 30], [900, 50, 40, 40]]
    d["sfa_boxes"] = [[100, 100, 50, 40], [100, 100, 50, 40], [300, 50, 0, 30],
                      [503, 200, 60, 60], [497, 200, 60, 60], [700, 100, 30, 30]]
    d["yolo_conf"] = [0.9, 0.9, 0.8, 0.5, 0.5, 0.31]
    d["sfa_conf"] = [0.9, 0.7, 0.8, 0.6, 0.6, 0.0]
    c["ties"] = d
    return c


def to_arrays(case):
    """Host arrays in the C-ABI layout for one frame."""
    yb = np.asarray(case["yolo_boxes"], np.int32).reshape(-1, 4)
    sb = np.asarray(case["sfa_boxes"], np.int32).reshape(-1, 4)
    return (yb, np.asarray(case["yolo_conf"], np.float64), np.asarray(case["yolo_cls"], np.int32),
            sb, np.asarray(case["sfa_conf"], np.float64))
