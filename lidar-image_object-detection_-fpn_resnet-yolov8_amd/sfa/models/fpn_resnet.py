"""Drop-in for the reference's models/fpn_resnet.py — KFPN ResNet on gfx950.

The module tree mirrors the reference's registration order exactly
(fpn_resnet.py:42-53 BasicBlock, :114-151 PoseResNet, heads in sorted() order
:135) so ``load_state_dict`` accepts the reference's 186-entry checkpoints and
``state_dict()`` round-trips them.  The submodules are parameter containers
only: ``PoseResNet.forward`` packs them (BatchNorm folded, OHWI layout) into one
device buffer on first use / after any parameter change, and runs the whole
forward — stem, 8 BasicBlocks, FPN, 15 heads, KFPN softmax — as HIP kernels
(libsfa_hip.so).  There is no CPU path: a CPU input raises ``SfaNativeError``.

Deviation (documented in DESIGN.md): the reference's per-forward visualisation
copies (fpn_resnet.py:189-242, ≈41 MB/frame) are opt-in through
``capture_visualization = True``.
"""

from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from sfa_hip import _lib
from sfa_hip import dropin as _dropin
from sfa_hip.runtime import KfpnEngine, pack_state_dict

BN_MOMENTUM = 0.1

# Generation of the module structure of the process: bumped whenever any module registers a
# parameter, buffer or submodule (torch's global registration hooks) and when PoseResNet._apply
# swaps tensors, so PoseResNet can keep its list of state tensors between forwards and re-walk
# state_dict() only when the structure may have changed (a state_dict walk is ~1.1 ms of host
# time per forward, the cached list's (data_ptr, _version) check ~40 us).
_STRUCT_GEN = [0]


def _bump_struct_gen(*_args, **_kw):
    _STRUCT_GEN[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_bump_struct_gen)
torch.nn.modules.module.register_module_buffer_registration_hook(_bump_struct_gen)
torch.nn.modules.module.register_module_module_registration_hook(_bump_struct_gen)

model_urls = {
    "resnet18": "https://download.pytorch.org/models/resnet18-5c106cde.pth",
}


def conv3x3(in_planes, out_planes, stride=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False)


class BasicBlock(nn.Module):
    """Parameter container of fpn_resnet.py:42-71 (executed fused by the HIP forward)."""

    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes, momentum=BN_MOMENTUM)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes, momentum=BN_MOMENTUM)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        raise RuntimeError("BasicBlock runs fused inside PoseResNet's HIP forward")


class PoseResNet(nn.Module):
    def __init__(self, block, layers, heads, head_conv, **kwargs):
        self.inplanes = 64
        self.deconv_with_bias = False
        self.heads = heads
        super().__init__()
        if block is not BasicBlock or list(layers) != [2, 2, 2, 2]:
            raise NotImplementedError("the HIP forward implements fpn_resnet_18 (BasicBlock x [2,2,2,2])")
        if head_conv != 64:
            raise NotImplementedError("the HIP forward implements head_conv = 64")
        self.head_conv = head_conv
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64, momentum=BN_MOMENTUM)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.conv_up_level1 = nn.Conv2d(768, 256, kernel_size=1, stride=1, padding=0)
        self.conv_up_level2 = nn.Conv2d(384, 128, kernel_size=1, stride=1, padding=0)
        self.conv_up_level3 = nn.Conv2d(192, 64, kernel_size=1, stride=1, padding=0)
        for fpn_idx, fpn_c in enumerate([256, 128, 64]):
            for head in sorted(self.heads):
                self.__setattr__(f"fpn{fpn_idx}_{head}", nn.Sequential(
                    nn.Conv2d(fpn_c, head_conv, kernel_size=3, padding=1, bias=True),
                    nn.ReLU(inplace=True),
                    nn.Conv2d(head_conv, self.heads[head], kernel_size=1, stride=1, padding=0)))
        # visualisation attributes (fpn_resnet.py:147-151); filled only when opted in
        self.capture_visualization = False
        self.kfpn_features = []
        self.fpn_outputs = {}
        self.kfpn_weights = {}
        self.backbone_features = {}
        self._arch = _lib.make_arch(dict(self.heads), head_conv)
        self._engines = {}
        self._sig = None
        self._state_tensors = None  # (structure generation, [state tensors]) cache of _signature

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * block.expansion, kernel_size=1, stride=stride, bias=False),
                nn.BatchNorm2d(planes * block.expansion, momentum=BN_MOMENTUM))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    # -------------------------------------------------------------- engine
    def _signature(self):
        """(data_ptr, version) of every state tensor: any in-place update, reload or move of a
        parameter changes it, and the engine repacks the weights."""
        cache = self._state_tensors
        if cache is None or cache[0] != _STRUCT_GEN[0]:
            cache = self._state_tensors = (_STRUCT_GEN[0], list(self.state_dict(keep_vars=True).values()))
        return tuple((t.data_ptr(), t._version) for t in cache[1])

    def _apply(self, fn, *args, **kw):  # .to() / .cuda() / .float() may replace the tensors
        out = super()._apply(fn, *args, **kw)
        _bump_struct_gen()
        return out

    def _engine(self, device) -> KfpnEngine:
        sig = self._signature()
        if sig != self._sig:
            self._engines = {}
            self._sig = sig
        eng = self._engines.get(device)
        if eng is None:
            packed = pack_state_dict(self.state_dict(), self._arch)
            eng = KfpnEngine(self._arch, packed, device)
            self._engines[device] = eng
        return eng

    def forward(self, x):
        return self.forward_layout(x, _lib.IN_NCHW3)

    def forward_layout(self, x, in_layout):
        """forward() with the input read as ``in_layout``: _lib.IN_NCHW3 (the reference's), or
        _lib.IN_NCHW3_FLIP_HW = forward(torch.flip(x, [2, 3])) with the flip fused in."""
        if not isinstance(x, torch.Tensor) or x.device.type != "cuda":
            raise _lib.SfaNativeError("PoseResNet.forward runs on the GPU (HIP) only; move the "
                                      "model input to a GPU device")
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected (B, 3, H, W), got {tuple(x.shape)}")
        if in_layout not in (_lib.IN_NCHW3, _lib.IN_NCHW3_FLIP_HW):
            raise ValueError(f"unsupported input layout {in_layout}")
        eng = self._engine(x.device)
        x = x.contiguous().float()
        with torch.no_grad(), torch.cuda.device(x.device):
            B, _, H, W = x.shape
            outs = eng.alloc_outputs(B, H, W)
            ws = eng.workspace(B, H, W)
            eng.forward_into(x, outs, in_layout, ws)
            if self.capture_visualization:
                self._capture(eng, ws, B, H, W)
            else:
                self.kfpn_features, self.fpn_outputs = [], {}
                self.kfpn_weights, self.backbone_features = {}, {}
        return outs

    def _capture(self, eng, ws, B, H, W):
        """Opt-in copies of the intermediate maps (fpn_resnet.py:189-242)."""
        views = eng.debug_views(ws, B, H, W)
        self.backbone_features = {k: views[k].clone() for k in ("layer1", "layer2", "layer3", "layer4")}
        self.kfpn_features = [views[k].clone() for k in ("up_level2", "up_level3", "up_level4")]
        self.fpn_outputs, self.kfpn_weights = {}, {}
        for name, lv in views["levels"].items():
            lv = [lv[0].repeat_interleave(2, 2).repeat_interleave(2, 3), lv[1], lv[2]]
            self.fpn_outputs[name] = [t.clone() for t in lv]
            self.kfpn_weights[name] = F.softmax(torch.stack(lv, dim=-1), dim=-1)

    def apply_kfpn(self, outs):
        raise RuntimeError("apply_kfpn runs fused inside the HIP forward (kfpn_combine kernel)")

    def get_visualization_data(self):
        return {"backbone_features": self.backbone_features, "kfpn_features": self.kfpn_features,
                "fpn_outputs": self.fpn_outputs, "kfpn_weights": self.kfpn_weights}

    def init_weights(self, num_layers, pretrained=True):
        if pretrained:
            raise RuntimeError("imagenet_pretrained=True downloads resnet weights "
                               "(fpn_resnet.py:283-286); no network access on this platform")


resnet_spec = {18: (BasicBlock, [2, 2, 2, 2])}


def get_pose_net(num_layers, heads, head_conv, imagenet_pretrained):
    if num_layers not in resnet_spec:
        raise NotImplementedError(f"fpn_resnet_{num_layers}: only 18 is implemented on gfx950")
    block_class, layers = resnet_spec[num_layers]
    model = PoseResNet(block_class, layers, heads, head_conv=head_conv)
    model.init_weights(num_layers, pretrained=imagenet_pretrained)
    return model


# names of the reference module this drop-in does not define come from the reference
__getattr__ = _dropin.module_getattr(__name__)
