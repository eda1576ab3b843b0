"""Drop-in for the reference's data_process/kitti_bev_utils.py.

``makeBEVMap(PointCloud_, boundary)`` (:22-55) keeps the reference contract —
numpy (N, 4) float32 points that already went through get_filtered_lidar in,
numpy (3, 608, 608) float64 out, channels [intensity, height, density] — but
the voxelisation runs on the GPU (sfa_bev_voxelize, bit-exact).
``makeBEVMap_device`` / ``makeBEVMapBatch`` keep everything on the device for
the fast path (raw sweeps in, NHWC4 or NCHW float32 out).

``get_corners`` / ``drawRotatedBox`` (:59-87) are OpenCV drawing helpers, kept
for API completeness (they need cv2 installed).
"""

from __future__ import annotations


import numpy as np
import torch

import config.kitti_config as cnf
from sfa_hip import _lib, runtime
from sfa_hip import dropin as _dropin


def makeBEVMap(PointCloud_, boundary, device=None):
    """Reference-compatible host API (float64 result)."""
    dev = runtime.host_api_device("makeBEVMap", device)
    pts = np.ascontiguousarray(PointCloud_, dtype=np.float32)
    if pts.ndim != 2 or pts.shape[1] != 4:
        raise ValueError(f"PointCloud_ must be (N, 4), got {pts.shape}")
    t = torch.from_numpy(pts).to(dev)
    out = runtime.voxelizer(dev)(t, [0, pts.shape[0]], boundary, layout=_lib.BEV_NCHW3_F64,
                                 flags=_lib.BEV_PREFILTERED)
    return out[0].cpu().numpy()


def makeBEVMap_device(points: torch.Tensor, boundary=None, raw: bool = True, layout: str = "nchw"):
    """One frame on the device: (N, 4) f32 GPU tensor -> (3, 608, 608) or (608, 608, 4) f32."""
    boundary = boundary or cnf.boundary
    lay = _lib.BEV_NHWC4_F32 if layout == "nhwc4" else _lib.BEV_NCHW3_F32
    out = runtime.voxelizer(points.device)(points, [0, points.shape[0]], boundary, layout=lay,
                                           flags=_lib.BEV_RAW if raw else _lib.BEV_PREFILTERED)
    return out[0]


def makeBEVMapBatch(points: torch.Tensor, offsets, boundary=None, raw: bool = True,
                    layout: str = "nhwc4"):
    """B frames packed back to back (offsets: B+1 ints) -> (B, 608, 608, 4) or (B, 3, 608, 608)."""
    boundary = boundary or cnf.boundary
    lay = _lib.BEV_NHWC4_F32 if layout == "nhwc4" else _lib.BEV_NCHW3_F32
    return runtime.voxelizer(points.device)(points, offsets, boundary, layout=lay,
                                            flags=_lib.BEV_RAW if raw else _lib.BEV_PREFILTERED)


def get_corners(x, y, w, l, yaw):
    """(4, 2) f32 BEV corners: front-left, rear-left, rear-right, front-right (:59-80)."""
    c, s = np.cos(yaw), np.sin(yaw)
    # (sign of w/2*cos, sign of l/2*sin) per corner; the y row uses (w/2*sin, l/2*cos)
    signs = ((-1, -1), (-1, 1), (1, 1), (1, -1))
    out = np.empty((4, 2), dtype=np.float32)
    for i, (sw, sl) in enumerate(signs):
        out[i, 0] = x + sw * w / 2 * c + sl * l / 2 * s
        out[i, 1] = y + sw * w / 2 * s - sl * l / 2 * c
    return out


def drawRotatedBox(img, x, y, w, l, yaw, color):
    import cv2  # drawing only (not on the device path)
    corners = get_corners(x, y, w, l, yaw).astype(int)
    cv2.polylines(img, [corners.reshape(-1, 1, 2)], True, color, 2)
    cv2.line(img, (corners[0, 0], corners[0, 1]), (corners[3, 0], corners[3, 1]), (255, 255, 0), 2)


# names of the reference module this drop-in does not define come from the reference
__getattr__ = _dropin.module_getattr(__name__)
