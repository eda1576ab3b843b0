"""FPN-ResNet-18 (KFPN) forward oracle in torch fp32 on CPU — TEST INFRASTRUCTURE ONLY.

A functional restatement of models/fpn_resnet.py that consumes a reference-format
state_dict (186 entries, names of fpn_resnet.py:114-151) and evaluates, in plain
torch CPU ops:

  stem           :120-123,179-182   conv7x7/s2/p3 -> BN(eps 1e-5) -> ReLU -> maxpool 3/2/1
  BasicBlock     :42-71             conv3x3(s)-BN-ReLU-conv3x3-BN (+downsample 1x1/s BN) + add, ReLU
  _make_layer    :153-167           resnet_spec[18] = [2, 2, 2, 2] (:289)
  FPN top-down   :197-210           bilinear x2 (align_corners=True) + cat + 1x1 conv (bias)
  heads          :133-145,219-233   per level & head: conv3x3(C->64, bias)-ReLU-conv1x1(64->c_h, bias);
                                    level 0 nearest-resized to H/4 x W/4
  apply_kfpn     :248-254           softmax over the 3 levels, sum(v * softmax(v))

It is both the numerics reference for the HIP conv path and the CPU baseline that
bench.py times on the GPU box's host cores (the reference Python cannot travel).
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

HEADS_DEFAULT = {"hm_cen": 3, "cen_offset": 2, "direction": 2, "z_coor": 1, "dim": 3}


def _bn(x, sd, p):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                        sd[p + ".bias"], False, 0.0, 1e-5)


def _block(x, sd, p, stride):
    out = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"], None, stride, 1), sd, p + ".bn1"))
    out = _bn(F.conv2d(out, sd[p + ".conv2.weight"], None, 1, 1), sd, p + ".bn2")
    if p + ".downsample.0.weight" in sd:
        res = _bn(F.conv2d(x, sd[p + ".downsample.0.weight"], None, stride, 0), sd, p + ".downsample.1")
    else:
        res = x
    return F.relu(out + res)


def forward(sd: dict, x: torch.Tensor, heads: dict = HEADS_DEFAULT, return_viz: bool = False):
    """sd: reference state_dict of torch CPU tensors; x: (B, 3, H, W) f32."""
    hm_h, hm_w = x.shape[2] // 4, x.shape[3] // 4
    y = F.relu(_bn(F.conv2d(x, sd["conv1.weight"], None, 2, 3), sd, "bn1"))
    y = F.max_pool2d(y, 3, 2, 1)
    feats = []
    for li, stride in zip(range(1, 5), (1, 2, 2, 2)):
        y = _block(y, sd, f"layer{li}.0", stride)
        y = _block(y, sd, f"layer{li}.1", 1)
        feats.append(y)
    l1, l2, l3, l4 = feats
    up1 = F.interpolate(l4, scale_factor=2, mode="bilinear", align_corners=True)
    c1 = F.conv2d(torch.cat((up1, l3), 1), sd["conv_up_level1.weight"], sd["conv_up_level1.bias"])
    up2 = F.interpolate(c1, scale_factor=2, mode="bilinear", align_corners=True)
    c2 = F.conv2d(torch.cat((up2, l2), 1), sd["conv_up_level2.weight"], sd["conv_up_level2.bias"])
    up3 = F.interpolate(c2, scale_factor=2, mode="bilinear", align_corners=True)
    up4 = F.conv2d(torch.cat((up3, l1), 1), sd["conv_up_level3.weight"], sd["conv_up_level3.bias"])
    ret, viz_w = {}, {}
    for head in heads:
        lv = []
        for idx, inp in enumerate((up2, up3, up4)):
            p = f"fpn{idx}_{head}"
            h = F.relu(F.conv2d(inp, sd[p + ".0.weight"], sd[p + ".0.bias"], 1, 1))
            h = F.conv2d(h, sd[p + ".2.weight"], sd[p + ".2.bias"])
            if h.shape[2] != hm_h or h.shape[3] != hm_w:
                h = F.interpolate(h, size=(hm_h, hm_w))
            lv.append(h)
        st = torch.stack(lv, dim=-1)
        w = F.softmax(st, dim=-1)
        ret[head] = (st * w).sum(dim=-1)
        viz_w[head] = w
    if return_viz:
        return ret, {"layer1": l1, "layer2": l2, "layer3": l3, "layer4": l4,
                     "kfpn": [up2, up3, up4], "kfpn_weights": viz_w}
    return ret


def state_dict_torch(sd_np: dict) -> dict:
    return {k: torch.from_numpy(v) for k, v in sd_np.items()}
