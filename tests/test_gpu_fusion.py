"""GPU parity of the fusion row (§8(f) #1): association, Bayesian / weighted fusion
and greedy NMS vs the reference functions' outputs — bit-exact (ints, f64)."""
import numpy as np
import pytest

import fusion_cases
from oracle import fusion_oracle as fo
from sfa_hip import _lib, runtime

pytestmark = pytest.mark.gpu
CASES = fusion_cases.cases()


def _frame(case):
    yb, yc, yk, sb, sc = fusion_cases.to_arrays(case)
    return (yb, yc, yk, sb, sc)


@pytest.mark.parametrize("mode,tag", [(_lib.FUSE_BAYES, "bayes"), (_lib.FUSE_WEIGHTED, "weighted")])
def test_fuse_batch_matches_reference(golden_fusion, gpu, mode, tag):
    names = list(CASES)
    # one launch for every case that shares thresholds with "typical"; run the rest alone
    for name in names:
        c = CASES[name]
        res = runtime.fuse_frames([_frame(c)], c["conf_thr"], c["fusion_iou"], c["nms_thr"], mode)[0]
        g = golden_fusion
        np.testing.assert_array_equal(res.boxes, g[f"{name}/{tag}/box"].reshape(-1, 4))
        np.testing.assert_array_equal(res.conf, g[f"{name}/{tag}/conf"])
        np.testing.assert_array_equal(res.cls, g[f"{name}/{tag}/cls"])
        np.testing.assert_array_equal(res.src, g[f"{name}/{tag}/src"])
        np.testing.assert_array_equal(res.boxes[res.keep], g[f"{name}/{tag}_nms/box"].reshape(-1, 4))
        np.testing.assert_array_equal(res.conf[res.keep], g[f"{name}/{tag}_nms/conf"])


def test_batched_frames_equal_single(gpu):
    same = [n for n, c in CASES.items() if (c["conf_thr"], c["fusion_iou"], c["nms_thr"]) == (0.3, 0.7, 0.5)]
    frames = [_frame(CASES[n]) for n in same]
    batch = runtime.fuse_frames(frames, 0.3, 0.7, 0.5)
    for n, r in zip(same, batch):
        fused, keep = fo.run(CASES[n], "bayes")
        np.testing.assert_array_equal(r.boxes, np.array([f[0] for f in fused], np.int64).reshape(-1, 4))
        np.testing.assert_array_equal(r.keep, np.array(keep, np.int64))


def test_iou_matrix_bit_exact(golden_fusion, gpu):
    for name, c in CASES.items():
        m = runtime.iou_matrix(c["yolo_boxes"], c["sfa_boxes"], gpu).cpu().numpy()
        np.testing.assert_array_equal(m, golden_fusion[f"{name}/iou"])


def test_random_frames_vs_oracle(gpu):
    rng = np.random.default_rng(17)
    frames, cases = [], []
    for f in range(64):
        ny, ns = int(rng.integers(0, 300)), int(rng.integers(0, 300))
        yb = np.stack([rng.integers(0, 1200, ny), rng.integers(0, 350, ny),
                       rng.integers(0, 120, ny), rng.integers(0, 90, ny)], 1)
        sb = yb[rng.integers(0, max(ny, 1), ns)] + rng.integers(-6, 7, (ns, 4)) if ny else \
            np.zeros((ns, 4), np.int64)
        sb = np.maximum(sb, 0)
        yc = rng.random(ny).astype(np.float32).astype(np.float64)
        sc = rng.random(ns)
        yk = rng.integers(0, 80, ny)
        frames.append((yb, yc, yk, sb, sc))
        cases.append(dict(yolo_boxes=yb.tolist(), yolo_conf=yc.tolist(), yolo_cls=yk.tolist(),
                          sfa_boxes=sb.tolist(), sfa_conf=sc.tolist(), conf_thr=0.3, fusion_iou=0.5,
                          nms_thr=0.4))
    for mode, mname in ((_lib.FUSE_BAYES, "bayes"), (_lib.FUSE_WEIGHTED, "weighted")):
        res = runtime.fuse_frames(frames, 0.3, 0.5, 0.4, mode)
        for r, c in zip(res, cases):
            fused, keep = fo.run(c, mname)
            np.testing.assert_array_equal(r.boxes, np.array([x[0] for x in fused], np.int64).reshape(-1, 4))
            np.testing.assert_array_equal(r.conf, np.array([x[1] for x in fused]))
            np.testing.assert_array_equal(r.src, np.array([x[3] for x in fused], np.int64))
            np.testing.assert_array_equal(r.keep, np.array(keep, np.int64))


def test_dict_api_matches_reference(golden_fusion, gpu):
    from utils import fusion_utils as fu
    g = golden_fusion
    for name, c in CASES.items():
        yd = (c["yolo_boxes"], c["yolo_conf"], c["yolo_cls"], fusion_cases.CLASS_NAMES)
        sd = (c["sfa_boxes"], c["sfa_conf"])
        for fn, tag in ((fu.create_fused_detections_wrapper, "bayes"), (fu.create_fused_detections, "weighted")):
            dets = fn(yd, sd, c["conf_thr"], c["fusion_iou"])
            np.testing.assert_array_equal(np.array([d["box"] for d in dets], np.int64).reshape(-1, 4),
                                          g[f"{name}/{tag}/box"].reshape(-1, 4))
            np.testing.assert_array_equal(np.array([d["confidence"] for d in dets]), g[f"{name}/{tag}/conf"])
            kept = fu.apply_nms_to_fused_detections(list(dets), c["nms_thr"])
            np.testing.assert_array_equal(np.array([d["box"] for d in kept], np.int64).reshape(-1, 4),
                                          g[f"{name}/{tag}_nms/box"].reshape(-1, 4))
    # the dict-level fusers on pre-filtered inputs
    c = CASES["low_fusion_thr"]
    ys, ss = fo.fuse_inputs(c["yolo_boxes"], c["yolo_conf"], c["yolo_cls"], c["sfa_boxes"],
                            c["sfa_conf"], c["conf_thr"])
    ydicts = [{"box": b, "confidence": cf, "class_id": k, "class_name": "x", "model": "YOLOv8"}
              for b, cf, k, _ in ys]
    sdicts = [{"box": b, "confidence": cf, "class_id": 0, "class_name": "car", "model": "SFA3D"}
              for b, cf, _, _ in ss]
    out = fu.bayesian_inspired_fuse_overlapping_detections(ydicts, sdicts, c["fusion_iou"])
    np.testing.assert_array_equal(np.array([d["box"] for d in out]), g["low_fusion_thr/bayes/box"])
    out = fu.fuse_overlapping_detections(ydicts, sdicts, c["fusion_iou"])
    np.testing.assert_array_equal(np.array([d["box"] for d in out]), g["low_fusion_thr/weighted/box"])
    assert fu.calculate_iou([0, 0, 10, 10], [5, 0, 10, 10]) == fo.iou([0, 0, 10, 10], [5, 0, 10, 10])


def test_gaussian_nms_matches_readme_snippet(golden_gaussian_nms, gpu):
    """sfa_gaussian_nms (all golden cases as frames of one launch) vs the README's gaussian_nms:
    the same products in the same order, so only the f64 exp of the device vs numpy can differ
    (last bit): relative tolerance 1e-14; boxes / order / count untouched by definition."""
    from conftest import gaussian_nms_case_names
    g = golden_gaussian_nms
    names = gaussian_nms_case_names(g)
    for sigma in sorted({float(g[f"{n}/sigma"]) for n in names}):
        sel = [n for n in names if float(g[f"{n}/sigma"]) == sigma]
        got = runtime.gaussian_nms_frames([(g[f"{n}/boxes"], g[f"{n}/conf_in"]) for n in sel], sigma, device=gpu)
        for n, c in zip(sel, got):
            ref = g[f"{n}/conf_out"]
            assert c.shape == ref.shape, n
            np.testing.assert_allclose(c, ref, rtol=1e-14, atol=0, err_msg=n)


def test_gaussian_nms_dropin_dicts_and_objects(golden_gaussian_nms, gpu):
    """utils.fusion_utils.gaussian_nms on the fusion dicts and on attribute objects (the
    README's form): in place, same order, same boxes."""
    from utils.fusion_utils import gaussian_nms
    g = golden_gaussian_nms
    boxes, conf = g["random130_sigma03/boxes"], g["random130_sigma03/conf_in"]
    ref = g["random130_sigma03/conf_out"]
    dets = [{"box": b.tolist(), "confidence": float(c), "class_id": 0} for b, c in zip(boxes, conf)]
    assert gaussian_nms(dets, sigma=0.3) is dets
    np.testing.assert_allclose([d["confidence"] for d in dets], ref, rtol=1e-14, atol=0)
    assert [d["box"] for d in dets] == boxes.tolist()

    class D:
        def __init__(self, b, c):
            self.box, self.confidence = b, c
    objs = [D(b.tolist(), float(c)) for b, c in zip(boxes, conf)]
    gaussian_nms(objs, sigma=0.3)
    np.testing.assert_allclose([o.confidence for o in objs], ref, rtol=1e-14, atol=0)
    assert gaussian_nms([], 0.5) == []
