"""Drop-in for the reference's data_process/kitti_data_utils.py (hot-path part).

``get_filtered_lidar(lidar, boundary, labels=None)`` (:228-251): the point
filter — inclusive box test on x, y, z in float32, then z -= minZ, input order
kept — runs as an order-preserving compaction on the GPU (sfa_filter_points).
Numpy in / numpy out like the reference; a GPU tensor in stays on the device.
The optional ``labels`` filter (:244-249, half-open on the max side) is a few
host comparisons on the label rows and stays on the host, as in the reference.

``Calibration`` (:94-173) — the KITTI calib-file reader the callers import beside the
filter (test.py:28, demo_front.py:36) — is host file parsing, restated here.  Every
other name of the reference module (label/heat-map helpers for training) resolves to the
reference's own module (``sfa_hip.dropin``).
"""

from __future__ import annotations

import numpy as np
import torch

from sfa_hip import dropin as _dropin
from sfa_hip import runtime


def get_filtered_lidar(lidar, boundary, labels=None):
    if isinstance(lidar, torch.Tensor):
        out = runtime.filter_points(lidar, boundary)
    else:
        pts = np.ascontiguousarray(lidar, dtype=np.float32)
        dev = runtime.host_api_device("get_filtered_lidar")
        out = runtime.filter_points(torch.from_numpy(pts).to(dev), boundary).cpu().numpy()
    if labels is None:
        return out
    return out, filter_labels(labels, boundary)


def filter_labels(labels, boundary):
    """The label half of get_filtered_lidar (:244-249): half-open box test on the label rows'
    x, y, z (host numpy, as the reference)."""
    minX, maxX = boundary["minX"], boundary["maxX"]
    minY, maxY = boundary["minY"], boundary["maxY"]
    minZ, maxZ = boundary["minZ"], boundary["maxZ"]
    keep = ((labels[:, 1] >= minX) & (labels[:, 1] < maxX) & (labels[:, 2] >= minY) &
            (labels[:, 2] < maxY) & (labels[:, 3] >= minZ) & (labels[:, 3] < maxZ))
    return labels[keep]


class Calibration(object):
    """KITTI calibration (kitti_data_utils.py:94-173): P2 / P3 (3x4), V2C = Tr_velo_to_cam
    (3x4), R0 = R_rect (3x3), all float32 as the reference parses them from lines 3-6 of
    the calib file (``name: v v v ...``), plus the intrinsics c_u, c_v, f_u, f_v, b_x, b_y."""

    def __init__(self, calib_filepath):
        calibs = self.read_calib_file(calib_filepath)
        self.P2 = np.reshape(calibs["P2"], [3, 4])
        self.P3 = np.reshape(calibs["P3"], [3, 4])
        self.V2C = np.reshape(calibs["Tr_velo2cam"], [3, 4])
        self.R0 = np.reshape(calibs["R_rect"], [3, 3])
        self.c_u = self.P2[0, 2]
        self.c_v = self.P2[1, 2]
        self.f_u = self.P2[0, 0]
        self.f_v = self.P2[1, 1]
        self.b_x = self.P2[0, 3] / (-self.f_u)
        self.b_y = self.P2[1, 3] / (-self.f_v)

    def read_calib_file(self, filepath):
        with open(filepath) as f:
            lines = f.readlines()

        def row(i, shape):
            vals = lines[i].strip().split(" ")[1:]
            return np.array(vals, dtype=np.float32).reshape(shape)

        return {"P2": row(2, (3, 4)), "P3": row(3, (3, 4)), "R_rect": row(4, (3, 3)),
                "Tr_velo2cam": row(5, (3, 4))}

    def cart2hom(self, pts_3d):
        """(N, 3 or 2) -> (N, 4 or 3): a column of float32 ones appended."""
        return np.hstack((pts_3d, np.ones((pts_3d.shape[0], 1), dtype=np.float32)))


__getattr__ = _dropin.module_getattr(__name__)
