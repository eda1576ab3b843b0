"""Camera-LiDAR fusion oracle (pure Python) — TEST INFRASTRUCTURE ONLY.

Restates the reference's fusion helpers (see tests/golden/gen_fusion_golden.py for
how they were run):

  iou                test6.py:76-101   [x, y, w, h] ints; 0 when the boxes are disjoint
                                       (strict '<' on the right/bottom edges) or the
                                       union is 0; int/int true division (correctly
                                       rounded, like IEEE f64 division of exact ints)
  associate_fuse     test6.py:231-308 (mode 'bayes'), test5.py:213-282 ('weighted'):
                     for every YOLO detection in order, the unmatched SFA box with the
                     largest IoU (> running max starting at 0, and >= threshold; ties ->
                     lower index) is fused; unmatched SFA boxes are appended in order
  fuse_inputs        test6.py:310-348 / test5.py:285-321: the conf >= threshold filter
  nms                test6.py:104-126: stable sort by confidence (descending), greedy,
                     suppress when IoU > threshold
  gaussian_nms       README.md:250-261 (the reference's only definition of it; no script
                     implements it): for i in order, every later detection j decays,
                     conf_j *= np.exp(-iou**2 / sigma); nothing is re-sorted or dropped
                     (pinned by tests/golden/gen_gaussian_nms_golden.py, which runs the
                     README's own snippet)
"""

from __future__ import annotations

import numpy as np

YOLO, SFA, FUSED = 0, 1, 2


def iou(a, b):
    x1, y1, w1, h1 = (int(v) for v in a)
    x2, y2, w2, h2 = (int(v) for v in b)
    xl, yt = max(x1, x2), max(y1, y2)
    xr, yb = min(x1 + w1, x2 + w2), min(y1 + h1, y2 + h2)
    if xr < xl or yb < yt:
        return 0.0
    inter = (xr - xl) * (yb - yt)
    union = w1 * h1 + w2 * h2 - inter
    return inter / union if union > 0 else 0.0


def _conf_to_var(c, vmax):
    return vmax * 100.0 if c < 0.1 else vmax * ((1.0 - c) / (c + 0.01))


def _gauss(m1, v1, m2, v2):
    v1, v2 = max(v1, 1e-6), max(v2, 1e-6)
    i1, i2 = 1.0 / v1, 1.0 / v2
    return (m1 * i1 + m2 * i2) / (i1 + i2)


def _fuse_box(mode, yb, yc, sb, sc):
    if mode == "bayes":
        out = []
        for k, vmax in enumerate((100.0, 100.0, 50.0, 50.0)):
            out.append(int(_gauss(yb[k], _conf_to_var(yc, vmax), sb[k], _conf_to_var(sc, vmax))))
        return out
    tot = yc + sc
    wy, ws = (0.5, 0.5) if tot == 0 else (yc / tot, sc / tot)
    return [int(wy * yb[k] + ws * sb[k]) for k in range(4)]


def fuse_inputs(yolo_boxes, yolo_conf, yolo_cls, sfa_boxes, sfa_conf, conf_thr):
    ys = [(list(b), float(c), int(k), YOLO) for b, c, k in zip(yolo_boxes, yolo_conf, yolo_cls)
          if c >= conf_thr]
    ss = [(list(b), float(c), 0, SFA) for b, c in zip(sfa_boxes, sfa_conf) if c >= conf_thr]
    return ys, ss


def associate_fuse(ys, ss, fusion_iou, mode="bayes"):
    matched = [False] * len(ss)
    out = []
    for yb, yc, ycls, _ in ys:
        best, best_iou = -1, 0.0
        for j, (sb, _sc, _k, _s) in enumerate(ss):
            if matched[j]:
                continue
            v = iou(yb, sb)
            if v > best_iou and v >= fusion_iou:
                best, best_iou = j, v
        if best >= 0:
            sb, sc = ss[best][0], ss[best][1]
            out.append((_fuse_box(mode, yb, yc, sb, sc), max(yc, sc), ycls, FUSED))
            matched[best] = True
        else:
            out.append((yb, yc, ycls, YOLO))
    out += [s for j, s in enumerate(ss) if not matched[j]]
    return out


def nms(dets, thr):
    order = sorted(range(len(dets)), key=lambda i: -dets[i][1])  # stable
    keep = []
    for i in order:
        if all(iou(dets[i][0], dets[k][0]) <= thr for k in keep):
            keep.append(i)
    return keep


def run(case, mode):
    ys, ss = fuse_inputs(case["yolo_boxes"], case["yolo_conf"], case["yolo_cls"],
                         case["sfa_boxes"], case["sfa_conf"], case["conf_thr"])
    fused = associate_fuse(ys, ss, case["fusion_iou"], mode)
    return fused, nms(fused, case["nms_thr"])


def gaussian_nms(boxes, conf, sigma=0.5):
    """README.md:250-261 on one frame: boxes [[x, y, w, h], ...], conf f64 -> decayed conf (list)."""
    c = [np.float64(v) for v in conf]
    n = len(c)
    for i in range(n):
        for j in range(i + 1, n):
            v = iou(boxes[i], boxes[j])
            c[j] = c[j] * np.exp(-v ** 2 / sigma)
    return [float(v) for v in c]
