"""Drop-in for the reference's utils/torch_utils.py (hot-path part).

``_sigmoid`` (:44-45) is in place — sigmoid then clamp(1e-4, 1 - 1e-4) — and
returns its argument, like the reference, for any strided float32 GPU tensor; it runs as a
HIP kernel (sfa_sigmoid_clamp_inplace) and refuses CPU tensors.
"""

from __future__ import annotations

import time

import torch

from sfa_hip import dropin as _dropin
from sfa_hip.runtime import sigmoid_clamp_


def _sigmoid(x):
    return sigmoid_clamp_(x)


def to_cpu(tensor):
    return tensor.detach().cpu()


def time_synchronized():
    """utils/misc.py:69-71."""
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return time.time()


# names of the reference module this drop-in does not define come from the reference
__getattr__ = _dropin.module_getattr(__name__)
