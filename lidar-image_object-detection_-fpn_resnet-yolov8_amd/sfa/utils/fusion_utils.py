"""Drop-in for the camera-LiDAR fusion helpers of the reference's fusion scripts
(test6.py:76-126,212-348; test5.py:213-321), on the GPU (sfa_fuse_detections).

The reference keeps these functions inside its scripts (which import ultralytics);
here they live in one module with the same names, arguments and dict outputs:
``{'box', 'confidence', 'class_id', 'class_name', 'model', 'color'}``.  The
association, fusion and NMS run as one wavefront per frame on the GPU, bit-identical
to the Python loops; ``fuse_frames`` batches many frames in one launch.  ``gaussian_nms``
is the Gaussian soft-NMS of the reference README (README.md:250-261; no reference script
defines it).
"""

from __future__ import annotations

import numpy as np
import torch

from sfa_hip import _lib, runtime

_MODEL = {_lib.SRC_YOLO: ("YOLOv8", (0, 255, 255)), _lib.SRC_LIDAR: ("SFA3D", (255, 0, 0))}
_FUSED_NAME = {_lib.FUSE_BAYES: "Fused (Bayesian-Inspired)", _lib.FUSE_WEIGHTED: "Fused (YOLOv8 + SFA3D)"}


def calculate_iou(box1, box2):
    return float(runtime.iou_matrix([box1], [box2])[0, 0].item())


def confidence_to_variance(confidence, max_variance_pixels=100.0, min_confidence_threshold=0.1):
    if confidence < min_confidence_threshold:
        return max_variance_pixels * 100.0
    return max_variance_pixels * ((1.0 - confidence) / (confidence + 0.01))


def fuse_gaussian_parameters(mean1, var1, mean2, var2):
    var1, var2 = max(var1, 1e-6), max(var2, 1e-6)
    i1, i2 = 1.0 / var1, 1.0 / var2
    return (mean1 * i1 + mean2 * i2) / (i1 + i2), 1.0 / (i1 + i2)


def _dicts(res, class_names, mode):
    out = []
    for box, conf, cls, src in zip(res.boxes, res.conf, res.cls, res.src):
        if src == _lib.SRC_FUSED:
            model, color = _FUSED_NAME[mode], (0, 255, 0)
        else:
            model, color = _MODEL[int(src)]
        name = class_names[int(cls)] if src != _lib.SRC_LIDAR else "car"
        out.append({"box": [int(v) for v in box], "confidence": float(conf), "class_id": int(cls),
                    "class_name": name, "model": model, "color": color})
    return out


def _run(yolov8_data, sfa3d_data, conf_thr, fusion_iou, mode, nms=None):
    yb, yc, yk, names = yolov8_data
    sb, sc = sfa3d_data
    res = runtime.fuse_frames([(np.asarray(yb).reshape(-1, 4), yc, yk, np.asarray(sb).reshape(-1, 4), sc)],
                              conf_thr, fusion_iou, 0.5 if nms is None else nms, mode,
                              apply_nms=nms is not None)[0]
    return res, names


def create_fused_detections_wrapper(yolov8_data, sfa3d_data, confidence_threshold, fusion_iou_threshold):
    """test6.py:310-348 (filter + Bayesian-inspired fusion)."""
    res, names = _run(yolov8_data, sfa3d_data, confidence_threshold, fusion_iou_threshold,
                      _lib.FUSE_BAYES)
    return _dicts(res, names, _lib.FUSE_BAYES)


def create_fused_detections(yolov8_data, sfa3d_data, confidence_threshold, fusion_iou_threshold):
    """test5.py:285-321 (filter + confidence-weighted fusion)."""
    res, names = _run(yolov8_data, sfa3d_data, confidence_threshold, fusion_iou_threshold,
                      _lib.FUSE_WEIGHTED)
    return _dicts(res, names, _lib.FUSE_WEIGHTED)


def apply_nms_to_fused_detections(detections, nms_threshold=0.5):
    """test6.py:104-126.  Returns the surviving dicts in NMS order (sorted by confidence)."""
    if len(detections) == 0:
        return []
    boxes = np.array([d["box"] for d in detections], np.int64).reshape(-1, 4)
    conf = np.array([d["confidence"] for d in detections], np.float64)
    # every entry goes in as an un-fusable "SFA" box (no YOLO side, no threshold): the
    # kernel's fused list is then the input list itself and `keep` indexes it
    res = runtime.fuse_frames([(np.zeros((0, 4)), np.zeros(0), np.zeros(0), boxes, conf)],
                              -np.inf, 2.0, nms_threshold, _lib.FUSE_BAYES, apply_nms=True)[0]
    return [detections[int(i)] for i in res.keep]


def gaussian_nms(detections, sigma=0.5):
    """README.md:250-261 gaussian_nms (Gaussian soft-NMS): for i in order, every later detection's
    confidence decays by exp(-iou**2 / sigma), in place; order and boxes unchanged, nothing is
    dropped. Detections are the fusion dicts (``'box'`` [x, y, w, h], ``'confidence'``) or objects
    with ``.box`` / ``.confidence`` (the README's attribute form); IoU is calculate_iou
    (test6.py:76-101). Runs on the GPU (sfa_gaussian_nms); returns ``detections``."""
    if len(detections) == 0:
        return detections
    as_dict = isinstance(detections[0], dict)
    get = (lambda d, k: d[k]) if as_dict else (lambda d, k: getattr(d, k))
    boxes = np.array([get(d, "box") for d in detections], np.int64).reshape(-1, 4)
    conf = np.array([get(d, "confidence") for d in detections], np.float64)
    out = runtime.gaussian_nms_frames([(boxes, conf)], sigma)[0]
    for d, c in zip(detections, out):
        if as_dict:
            d["confidence"] = float(c)
        else:
            d.confidence = float(c)
    return detections


def _fuse_dicts(yolov8_detections, sfa3d_detections, thr, mode):
    res = runtime.fuse_frames([(np.asarray([d["box"] for d in yolov8_detections]).reshape(-1, 4),
                                [d["confidence"] for d in yolov8_detections],
                                [d["class_id"] for d in yolov8_detections],
                                np.asarray([d["box"] for d in sfa3d_detections]).reshape(-1, 4),
                                [d["confidence"] for d in sfa3d_detections])],
                              -np.inf, thr, 0.5, mode, apply_nms=False)[0]
    out = []
    for box, conf, src, org in zip(res.boxes, res.conf, res.src, res.origin):
        if src == _lib.SRC_FUSED:
            d = dict(yolov8_detections[int(org)])
            d.update(box=[int(v) for v in box], confidence=float(conf), model=_FUSED_NAME[mode],
                     color=(0, 255, 0))
            out.append(d)
        elif src == _lib.SRC_YOLO:
            out.append(yolov8_detections[int(org)])
        else:
            out.append(sfa3d_detections[int(org)])
    return out


def bayesian_inspired_fuse_overlapping_detections(yolov8_detections, sfa3d_detections,
                                                  fusion_iou_threshold):
    """test6.py:231-308 on already-filtered detection dicts."""
    return _fuse_dicts(yolov8_detections, sfa3d_detections, fusion_iou_threshold, _lib.FUSE_BAYES)


def fuse_overlapping_detections(yolov8_detections, sfa3d_detections, fusion_iou_threshold):
    """test5.py:213-282 on already-filtered detection dicts."""
    return _fuse_dicts(yolov8_detections, sfa3d_detections, fusion_iou_threshold, _lib.FUSE_WEIGHTED)


def fuse_frames(frames, confidence_threshold=0.3, fusion_iou_threshold=0.7, nms_threshold=0.5,
                weighted=False):
    """Batched form: many frames in one launch -> list of runtime.FusionResult."""
    return runtime.fuse_frames(frames, confidence_threshold, fusion_iou_threshold, nms_threshold,
                               _lib.FUSE_WEIGHTED if weighted else _lib.FUSE_BAYES, apply_nms=True)


def convert_sfa3d_to_2d_boxes(sfa_detections, calib, img_shape, device=None):
    """test6.py:129-187: post_processing's per-class dict -> (list of int [x, y, w, h] image
    boxes, list of confidences).  As in the reference the "confidence" is column 0 of
    convert_det_to_real_values, i.e. the class id, so class 0 rows never pass the 0.3 cut.
    The metres conversion is the host API (evaluation_utils.py:177-193); the camera
    transform, corner projection and clipping run on the GPU (sfa_project_boxes).
    ``calib`` needs the Calibration attributes V2C (3x4), R0 (3x3), P2 (3x4)."""
    from utils.evaluation_utils import convert_det_to_real_values
    real = np.asarray(convert_det_to_real_values(sfa_detections), np.float64).reshape(-1, 8)
    if len(real) == 0:
        return [], []
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    off = torch.tensor([0, len(real)], dtype=torch.int32, device=dev)
    cal = runtime.make_calib(calib.V2C, calib.R0, calib.P2, img_shape)
    boxes, conf, _, _, boff = runtime.project_boxes(torch.from_numpy(real).to(dev), off, [cal])
    n = int(boff[1].item())
    return ([[int(v) for v in b] for b in boxes[:n].cpu().numpy()],
            [float(c) for c in conf[:n].cpu().numpy()])
