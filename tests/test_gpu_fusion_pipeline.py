"""BASELINE config #5 chain on the GPU (runtime.FusionPipeline): sweeps -> BEV -> forward ->
decode -> post_process -> camera boxes -> fusion + NMS, checked stage by stage against the
oracles (tests/test_project_oracle.py and tests/test_fusion_oracle.py pin those against the
reference) on the pipeline's own decoded detections.  Camera boxes are synthetic (YOLOv8n is
not available: parity unpinned for the camera detector itself)."""
import numpy as np
import pytest
import torch

import golden_cases as gc
import project_cases
from oracle import fusion_oracle as fo
from oracle import project_oracle as po
from sfa_hip import _lib, runtime, synthetic

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("conf_source,nms", [(_lib.CONF_CLASS_ID, "greedy"), (_lib.CONF_SCORE, "greedy"),
                                             (_lib.CONF_SCORE, "gaussian")])
def test_fusion_pipeline_matches_oracles(golden, gpu, conf_source, nms):
    """nms="gaussian": the README's Gaussian soft-NMS (README.md:250-261) on the fused lists
    instead of the greedy NMS: confidences within 1e-14 rel. of the oracle (device vs numpy exp)."""
    B = 8  # BASELINE configs[4] batch
    arch = _lib.make_arch(gc.HEADS)
    eng = runtime.KfpnEngine(arch, runtime.pack_state_dict(gc.state_dict_np(golden.model), arch), gpu)
    cal = project_cases.calibs()
    names = ["avg", "seq"] * (B // 2)
    calibs = [runtime.make_calib(cal[n]["V2C"], cal[n]["R0"], cal[n]["P2"], cal[n]["img_shape"])
              for n in names]
    clouds = [synthetic.synthetic_point_cloud(s) for s in range(1, B + 1)]
    fp = runtime.FusionPipeline(eng, B, calibs, K=50, max_points=sum(c.shape[0] for c in clouds),
                                conf_source=conf_source, fusion_iou_threshold=0.3, nms=nms, soft_nms_sigma=0.5)
    fp.set_points(clouds)
    # camera boxes: jittered copies of the first pass's projected boxes + random extras
    fp.set_camera([(np.zeros((0, 4)), np.zeros(0), np.zeros(0))] * B)
    fp.run()
    soff = fp.soff.cpu().numpy()
    sb = fp.sboxes.cpu().numpy()
    rng = np.random.default_rng(11)
    cams = []
    for b in range(B):
        base = sb[soff[b]:soff[b + 1]]
        jit = rng.integers(-3, 4, base.shape)
        extra = np.stack([rng.integers(0, 1200, 6), rng.integers(0, 350, 6),
                          rng.integers(5, 80, 6), rng.integers(5, 60, 6)], 1)
        boxes = np.concatenate([np.maximum(base + jit, 0), extra]).astype(np.int64)
        conf = rng.random(len(boxes)).astype(np.float32).astype(np.float64)
        cls = rng.integers(0, 80, len(boxes))
        cams.append((boxes, conf, cls))
    fp.set_camera(cams)
    fp.capture()
    fp.replay()
    torch.cuda.synchronize()
    res = fp.results()
    dets = fp.det.dets.cpu().numpy()
    n_fused = 0
    for b in range(B):
        preds = po.post_frame(dets[b])
        real = po.real_rows(preds)
        sc = np.concatenate([preds[j][:, 0] for j in range(3)]).astype(np.float64)
        ob, oc, _, _ = po.image_boxes(real, cal[names[b]], cal[names[b]]["img_shape"], 0.3,
                                      sc if conf_source == _lib.CONF_SCORE else None)
        boxes, conf, cls = cams[b]
        case = dict(yolo_boxes=boxes.tolist(), yolo_conf=conf.tolist(), yolo_cls=cls.tolist(),
                    sfa_boxes=ob.tolist(), sfa_conf=oc.tolist(), conf_thr=0.3, fusion_iou=0.3,
                    nms_thr=0.5)
        fused, keep = fo.run(case, "bayes")
        gb, gconf, gcls, gsrc, gkeep = res[b]
        np.testing.assert_array_equal(gb, np.array([f[0] for f in fused], np.int64).reshape(-1, 4))
        np.testing.assert_array_equal(gsrc, np.array([f[3] for f in fused]))
        if nms == "gaussian":
            ref = fo.gaussian_nms([f[0] for f in fused], [f[1] for f in fused], 0.5)
            np.testing.assert_allclose(gconf, np.array(ref, np.float64).reshape(-1), rtol=1e-14, atol=0)
            np.testing.assert_array_equal(gkeep, np.arange(len(fused)))
        else:
            np.testing.assert_array_equal(gconf, np.array([f[1] for f in fused]))
            np.testing.assert_array_equal(gkeep, np.array(keep))
        n_fused += int(np.sum(gsrc == _lib.SRC_FUSED))
    if conf_source == _lib.CONF_SCORE:
        assert n_fused > 0
