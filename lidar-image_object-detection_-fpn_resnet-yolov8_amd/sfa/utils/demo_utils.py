"""Drop-in for the detection step of the reference demos (utils/demo_utils.py:109-127
``do_detect``, used by demo_front.py and demo_2_sides.py).

The forward, sigmoid and decode run as HIP kernels; the back view's
``torch.flip(bevmap, [1, 2])`` (demo_utils.py:110-111) is fused into the model's input
layout conversion (``SFA_IN_NCHW3_FLIP_HW``), so the GPU reads the unflipped map.  The
flipped map is still returned for drawing, as the reference returns it.  The dataset
download helpers (wget, network) are not part of the hot path and are not provided.
"""

from __future__ import annotations

import time

import numpy as np
import torch

from sfa_hip import _lib
from utils.evaluation_utils import decode, post_processing
from utils.torch_utils import _sigmoid


def time_synchronized():
    torch.cuda.synchronize() if torch.cuda.is_available() else None
    return time.time()


def do_detect(configs, model, bevmap, is_front):
    """demo_utils.py:109-127: (detections of the frame, the (flipped) bevmap, fps)."""
    dev = configs.device
    x = bevmap.unsqueeze(0).to(dev, non_blocking=True).float()
    t1 = time_synchronized()
    if is_front:
        outputs = model(x)
    else:
        outputs = model.forward_layout(x, _lib.IN_NCHW3_FLIP_HW)
    outputs["hm_cen"] = _sigmoid(outputs["hm_cen"])
    outputs["cen_offset"] = _sigmoid(outputs["cen_offset"])
    detections = decode(outputs["hm_cen"], outputs["cen_offset"], outputs["direction"],
                        outputs["z_coor"], outputs["dim"], K=configs.K)
    detections = detections.cpu().numpy().astype(np.float32)
    detections = post_processing(detections, configs.num_classes, configs.down_ratio,
                                 configs.peak_thresh)
    t2 = time_synchronized()
    if not is_front:
        bevmap = torch.flip(bevmap, [1, 2])  # the returned display copy, as the reference
    return detections[0], bevmap, 1 / max(t2 - t1, 1e-9)
