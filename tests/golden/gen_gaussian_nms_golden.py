#!/usr/bin/env python3
"""Golden fixtures for the Gaussian soft-NMS (BASELINE north_star "Gaussian ... NMS"), made by
running the REFERENCE's own definition of it in the build container.

The reference defines gaussian_nms only in its README (README.md:250-261, the "### 2. Gaussian
NMS" python block); no script implements it (north-star note 1).  This script reads
that block from /root/reference/README.md at run time, extracts the function with ``ast`` and
executes it unchanged.  The snippet's call-site conventions are supplied around it: detections
are objects with ``.box`` ([x, y, w, h] ints, as the fusion scripts' boxes) and ``.confidence``,
and its ``calculate_iou(det, other_det)`` is test6.py:76-101 calculate_iou (also extracted with
``ast``) applied to the two boxes.  Inputs are seeded; inputs and outputs go to
tests/golden/gaussian_nms_golden.npz.

Why the reference's text is executed rather than oracle/fusion_oracle.gaussian_nms (advisor note,
round 2): the fixtures pin the oracle; generated from the oracle they would pin nothing.  Only the
two named FunctionDef nodes are compiled (no module-level statement of the README block or of
test6.py runs), in a namespace holding numpy alone, in the build container, by hand — never by a
test, smoke() or bench.py.
"""

from __future__ import annotations

import ast
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def readme_gaussian_nms():
    text = open(os.path.join(REF, "README.md")).read()
    m = re.search(r"### 2\. Gaussian NMS\s*```python\n(.*?)```", text, re.S)
    assert m, "README Gaussian NMS block not found"
    return m.group(1)


def extract_fn(src, name, ns, filename):
    tree = ast.parse(src, filename=filename)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name]
    assert len(keep) == 1, (filename, name)
    exec(compile(ast.Module(body=keep, type_ignores=[]), filename, "exec"), ns)
    return ns[name]


class Det:
    def __init__(self, box, confidence):
        self.box = [int(v) for v in box]
        self.confidence = confidence


def cases():
    """name -> (boxes (n, 4) int32, conf (n,) f64, sigma)."""
    rng = np.random.default_rng(20261016)
    out = {}

    def rand_boxes(n, spread, wmax):
        xy = rng.integers(0, spread, size=(n, 2))
        wh = rng.integers(1, wmax, size=(n, 2))
        return np.concatenate([xy, wh], 1).astype(np.int32)

    out["empty"] = (np.zeros((0, 4), np.int32), np.zeros(0), 0.5)
    out["single"] = (np.array([[10, 20, 30, 40]], np.int32), np.array([0.9]), 0.5)
    out["identical_pair"] = (np.array([[10, 20, 30, 40]] * 2, np.int32), np.array([0.8, 0.7]), 0.5)
    out["disjoint"] = (np.array([[i * 50, 0, 40, 40] for i in range(5)], np.int32), rng.random(5), 0.5)
    out["touching_edges"] = (np.array([[0, 0, 10, 10], [10, 0, 10, 10], [0, 10, 10, 10], [5, 5, 0, 0]],
                                      np.int32), np.array([0.9, 0.8, 0.7, 0.6]), 0.5)
    out["random40"] = (rand_boxes(40, 300, 120), rng.random(40), 0.5)
    out["random130_sigma03"] = (rand_boxes(130, 400, 150), rng.random(130), 0.3)
    out["clustered300_sigma1"] = (rand_boxes(300, 120, 80), rng.random(300), 1.0)
    sort_conf = np.sort(rng.random(64))[::-1].copy()
    out["sorted64"] = (rand_boxes(64, 200, 100), sort_conf, 0.5)
    return out


def main():
    ns = {"np": np}
    t6 = open(os.path.join(REF, "test6.py")).read()
    ref_iou = extract_fn(t6, "calculate_iou", {"np": np}, "test6.py")
    ns["calculate_iou"] = lambda a, b: ref_iou(a.box, b.box)  # the snippet's call convention
    gaussian_nms = extract_fn(readme_gaussian_nms(), "gaussian_nms", ns, "README.md")
    arrays = {}
    for name, (boxes, conf, sigma) in cases().items():
        dets = [Det(b, float(c)) for b, c in zip(boxes, conf)]
        gaussian_nms(dets, sigma=sigma)
        arrays[f"{name}/boxes"] = boxes
        arrays[f"{name}/conf_in"] = np.asarray(conf, np.float64)
        arrays[f"{name}/sigma"] = np.float64(sigma)
        arrays[f"{name}/conf_out"] = np.array([d.confidence for d in dets], np.float64)
    np.savez_compressed(os.path.join(HERE, "gaussian_nms_golden.npz"), **arrays)
    print(f"wrote {len(arrays) // 4} cases")


if __name__ == "__main__":
    main()
