"""Drop-in for the reference's data_process/kitti_data_utils.py (hot-path part).

``get_filtered_lidar(lidar, boundary, labels=None)`` (:228-251): the point
filter — inclusive box test on x, y, z in float32, then z -= minZ, input order
kept — runs as an order-preserving compaction on the GPU (sfa_filter_points).
Numpy in / numpy out like the reference; a GPU tensor in stays on the device.
The optional ``labels`` filter (:244-249, half-open on the max side) is a few
host comparisons on the label rows and stays on the host, as in the reference.
"""

from __future__ import annotations

import numpy as np
import torch

from sfa_hip import runtime


def get_filtered_lidar(lidar, boundary, labels=None):
    if isinstance(lidar, torch.Tensor):
        out = runtime.filter_points(lidar, boundary)
    else:
        if not torch.cuda.is_available():
            raise runtime.SfaNativeError("get_filtered_lidar runs on the GPU (HIP); no GPU visible")
        pts = np.ascontiguousarray(lidar, dtype=np.float32)
        dev = torch.device("cuda", torch.cuda.current_device())
        out = runtime.filter_points(torch.from_numpy(pts).to(dev), boundary).cpu().numpy()
    if labels is None:
        return out
    minX, maxX = boundary["minX"], boundary["maxX"]
    minY, maxY = boundary["minY"], boundary["maxY"]
    minZ, maxZ = boundary["minZ"], boundary["maxZ"]
    keep = ((labels[:, 1] >= minX) & (labels[:, 1] < maxX) & (labels[:, 2] >= minY) &
            (labels[:, 2] < maxY) & (labels[:, 3] >= minZ) & (labels[:, 3] < maxZ))
    return out, labels[keep]
