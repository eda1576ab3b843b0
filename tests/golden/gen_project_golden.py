#!/usr/bin/env python3
"""Golden fixtures for on-device post-processing + camera projection,
made by running the REFERENCE's own functions in the build container:

  utils/evaluation_utils.py:112-163   post_processing (one frame per call: it returns
                                      only the last frame's dict, :158)
  utils/evaluation_utils.py:177-193   convert_det_to_real_values
  data_process/transformation.py:99-107 lidar_to_camera_box
  test6.py:129-187                    convert_sfa3d_to_2d_boxes (extracted with ast —
                                      test6.py imports ultralytics at module top)

The sfa/ modules are imported with gen_golden.py's recipe (scratch copy under /tmp named
``sfa``, stub cv2).  Inputs come from tests/project_cases.py plus the end-to-end
detections already in model_golden.npz.  Output: tests/golden/project_golden.npz.
"""

from __future__ import annotations

import ast
import contextlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, HERE)
import gen_golden  # noqa: E402
import project_cases  # noqa: E402

REF = gen_golden.REF


class _Calib:
    def __init__(self, d):
        self.V2C, self.R0, self.P2 = d["V2C"], d["R0"], d["P2"]


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not present")
    ref = gen_golden._import_reference()
    from data_process import transformation  # the scratch copy imported above
    tree = ast.parse(open(os.path.join(REF, "test6.py")).read())
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "convert_sfa3d_to_2d_boxes"]
    assert len(fn) == 1
    ns = {"np": np, "convert_det_to_real_values": ref["ev"].convert_det_to_real_values,
          "lidar_to_camera_box": transformation.lidar_to_camera_box}
    exec(compile(ast.Module(body=fn, type_ignores=[]), "test6.py", "exec"), ns)
    to2d = ns["convert_sfa3d_to_2d_boxes"]

    cals = project_cases.calibs()
    cases = project_cases.cases()
    mg = np.load(os.path.join(HERE, "model_golden.npz"))
    cases["e2e"] = (mg["e2e/dets"].astype(np.float32), ["avg"])
    res = {}
    for name, (dets, cal_names) in cases.items():
        res[f"{name}/dets"] = dets
        res[f"{name}/calibs"] = np.array(cal_names)
        for b in range(dets.shape[0]):
            with contextlib.redirect_stdout(io.StringIO()):
                post = ref["ev"].post_processing(dets[b:b + 1].copy(), 3, 4, 0.2)[0]
            real = ref["ev"].convert_det_to_real_values(post)
            real = np.asarray(real, np.float64).reshape(-1, 8)
            cal = cals[cal_names[b]]
            cam = transformation.lidar_to_camera_box(real[:, 1:], cal["V2C"], cal["R0"], cal["P2"]) \
                if len(real) else np.zeros((0, 7))
            boxes, conf = to2d(post, _Calib(cal), cal["img_shape"])
            k = f"{name}/{b}"
            for j in range(3):
                res[f"{k}/post{j}"] = post[j]
            res[f"{k}/real"] = real
            res[f"{k}/cam"] = np.asarray(cam, np.float64).reshape(-1, 7)
            res[f"{k}/boxes"] = np.array(boxes, np.int64).reshape(-1, 4)
            res[f"{k}/conf"] = np.array(conf, np.float64)
            print(f"project {name}/{b}: rows {len(real)}, boxes {len(boxes)}")
    for n, cal in cals.items():
        for f in ("V2C", "R0", "P2"):
            res[f"calib/{n}/{f}"] = cal[f]
        res[f"calib/{n}/img_shape"] = np.array(cal["img_shape"])
    np.savez_compressed(os.path.join(HERE, "project_golden.npz"), **res)


if __name__ == "__main__":
    main()
