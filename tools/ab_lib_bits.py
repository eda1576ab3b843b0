"""Bit-comparison of two builds of libsfa_hip.so on the same forwards (round-4 prune check).

    SFA_HIP_LIB=<lib> [SFA_ABI_EXPECT=1] python tools/ab_lib_bits.py run out.npz
    python tools/ab_lib_bits.py compare a.npz b.npz

`run` packs the synthetic weights, runs the fp16x3 forward (default options) at a few sizes that
cover every kernel path of the bench (608 x 608 with 10 frames: r3 heads, strip convs, r3 body
convs, FPN skip convs, split-K layer4, the patch stem) and saves every head map; `compare`
asserts the two files are bit-identical."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lidar-image_object-detection_-fpn_resnet-yolov8_amd", "sfa"))

CASES = [(2, 96, 96), (3, 160, 192), (10, 608, 608)]


def run(out):
    import torch
    from sfa_hip import _lib, runtime, synthetic
    _lib.ABI_VERSION = int(os.environ.get("SFA_ABI_EXPECT", _lib.ABI_VERSION))
    import ctypes
    probe = ctypes.CDLL(_lib.LIB_PATH)  # an older build lacks the newer entry points: bind what it has
    for name in [n for n in _lib._PROTOS if not hasattr(probe, n)]:
        print("not in", _lib.LIB_PATH, ":", name)
        del _lib._PROTOS[name]
    dev = torch.device("cuda", 0)
    arch = _lib.make_arch(runtime.DEFAULT_HEADS)
    sd = synthetic.synthetic_state_dict(_lib.state_layout(arch), 0)
    eng = runtime.KfpnEngine(arch, runtime.pack_state_dict(sd, arch), dev, math=_lib.MATH_FP16X3)
    res = {}
    for B, H, W in CASES:
        x = torch.from_numpy(synthetic.synthetic_bev(B, H, W, seed=B + H)).to(dev)
        o = eng.forward(x)
        for h, v in o.items():
            res[f"{B}x{H}x{W}/{h}"] = v.cpu().numpy()
    np.savez(out, **res)
    print("saved", out, len(res))


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    assert sorted(A.files) == sorted(Bz.files)
    bad = [k for k in A.files if not np.array_equal(A[k], Bz[k])]
    for k in bad:
        d = np.abs(A[k] - Bz[k])
        print("DIFF", k, float(d.max()))
    print("bit-identical" if not bad else f"{len(bad)} of {len(A.files)} maps differ")
    return 0 if not bad else 1


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
