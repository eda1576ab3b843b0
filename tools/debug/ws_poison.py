"""Does any forward kernel read workspace bytes it has not written?  The bs=16 608x608 fp16x3
forward on workspaces / head outputs pre-filled with different byte patterns; every head map and
intermediate must be bit-identical to the zero-filled run.  (GPU box: python tools/debug/ws_poison.py)"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lidar-image_object-detection_-fpn_resnet-yolov8_amd", "sfa"))
from sfa_hip import _lib, runtime, synthetic  # noqa: E402

B, H, W = int(os.environ.get("B", 16)), int(os.environ.get("H", 608)), int(os.environ.get("W", 608))
dev = torch.device("cuda", 0)
arch = _lib.make_arch(runtime.DEFAULT_HEADS)
sd = synthetic.synthetic_state_dict(_lib.state_layout(arch), 0)
eng = runtime.KfpnEngine(arch, runtime.pack_state_dict(sd, arch), dev)
if os.environ.get("SIDE", "1") == "0":
    eng.set_side_streams(False)
x = torch.from_numpy(synthetic.synthetic_bev(B, H, W, seed=1)).to(dev)
nb = eng.workspace_bytes(B, H, W)


def run(byte):
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    if byte == "rand":
        g = torch.Generator(device=dev).manual_seed(5)
        ws.copy_(torch.randint(0, 256, (nb,), dtype=torch.uint8, device=dev, generator=g))
    else:
        ws.fill_(byte)
    outs = eng.alloc_outputs(B, H, W)
    for v in outs.values():
        v.view(torch.uint8).fill_(0x7F if byte != 0 else 0)
    eng.forward_into(x, outs, workspace=ws)
    torch.cuda.synchronize()
    v = eng.debug_views(ws, B, H, W)
    res = {k: outs[k].cpu().numpy() for k in outs}
    for k in ("layer1", "layer2", "layer3", "layer4", "up_level2", "up_level3", "up_level4"):
        res[k] = v[k].cpu().numpy()
    for h, lv in v["levels"].items():
        for j, t in enumerate(lv):
            res[f"L{j}/{h}"] = t.cpu().numpy()
    return res


ref = run(0)
again = run(0)
print("zero vs zero:", [k for k in ref if not np.array_equal(ref[k], again[k])])
for byte in (0xFF, 0x7F, 0x3C, "rand"):
    r = run(byte)
    bad = [k for k in ref if not np.array_equal(ref[k], r[k], equal_nan=True)]
    print("fill", byte, "differs:", bad)
    for k in bad[:6]:
        d = np.abs(np.nan_to_num(ref[k].astype(np.float64)) - np.nan_to_num(r[k].astype(np.float64)))
        where = np.argwhere(~np.isclose(ref[k], r[k], rtol=0, atol=0, equal_nan=True))
        print("   ", k, "max", float(d.max()), "n", int(len(where)), "first", where[:3].tolist(),
              "frames", sorted(set(where[:, 0].tolist()))[:20])
