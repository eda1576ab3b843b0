"""Drop-in for the reference's models/model_utils.py (create_model, :25-43).

``create_model(configs)`` reads ``configs.arch`` ('fpn_resnet_18'), ``.heads``
(dict; insertion order = forward output order), ``.head_conv`` and
``.imagenet_pretrained`` exactly as the reference does and returns the
HIP-backed ``PoseResNet``.  Error behaviour follows the reference: a bad arch
suffix raises ``ValueError`` (:27-31), an unknown backbone fails an assertion
(:41).  The plain ``resnet_*`` arch (models/resnet.py) is not part of this
hot path and raises ``NotImplementedError``.
"""

from __future__ import annotations

from models import fpn_resnet
from sfa_hip import dropin as _dropin


def create_model(configs):
    try:
        num_layers = int(configs.arch.split("_")[-1])
    except Exception:
        raise ValueError
    if "fpn_resnet" in configs.arch:
        print("using ResNet architecture with feature pyramid")
        return fpn_resnet.get_pose_net(num_layers=num_layers, heads=configs.heads,
                                       head_conv=configs.head_conv,
                                       imagenet_pretrained=configs.imagenet_pretrained)
    if "resnet" in configs.arch:
        raise NotImplementedError("plain resnet_* (models/resnet.py) is outside the gfx950 hot path")
    assert False, "Undefined model backbone"


def get_num_parameters(model):
    m = model.module if hasattr(model, "module") else model
    return sum(p.numel() for p in m.parameters() if p.requires_grad)


# names of the reference module this drop-in does not define come from the reference
__getattr__ = _dropin.module_getattr(__name__)
