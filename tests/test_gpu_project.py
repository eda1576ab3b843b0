"""GPU parity of on-device post-processing + camera projection:
sfa_post_process (post_processing + convert_det_to_real_values, every frame) and
sfa_project_boxes (convert_sfa3d_to_2d_boxes) vs the reference's outputs and the oracle.

Tolerances (stated, everything else is bit-exact):
* yaw (atan2) — numpy's f32 arctan2 is a SIMD approximation (<= 3 ulp on AVX-512), the
  kernel rounds an f64 atan2: <= 4 f32 ulp vs the fixtures, <= 1 ulp vs f32(atan2 f64).
* projected extents (f64) — BLAS summation order / libm sin-cos: rtol 1e-12 vs the oracle;
  the int boxes themselves must be identical.
"""
import numpy as np
import pytest
import torch

from oracle import project_oracle as po
from sfa_hip import _lib, runtime

pytestmark = pytest.mark.gpu
YAW_ULP = 4


def _ulp(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


def _calibs(g, names):
    out, shapes = [], []
    for n in names:
        n = str(n)
        shape = tuple(int(v) for v in g[f"calib/{n}/img_shape"])
        out.append(runtime.make_calib(g[f"calib/{n}/V2C"], g[f"calib/{n}/R0"], g[f"calib/{n}/P2"],
                                      shape))
        shapes.append(({f: g[f"calib/{n}/{f}"] for f in ("V2C", "R0", "P2")}, shape))
    return out, shapes


def _split(t, off):
    t, off = t.cpu().numpy(), off.cpu().numpy()
    return [t[off[b]:off[b + 1]] for b in range(len(off) - 1)]


@pytest.mark.parametrize("name", ["typical", "edges", "e2e"])
def test_post_process_matches_reference(golden_project, gpu, name):
    g = golden_project
    dets = torch.from_numpy(g[f"{name}/dets"]).to(gpu)
    preds, real, off = runtime.post_process(dets)
    P, R = _split(preds, off), _split(real, off)
    for b in range(dets.shape[0]):
        ref = np.concatenate([g[f"{name}/{b}/post{j}"] for j in range(3)]).reshape(-1, 8)
        assert P[b].shape == ref.shape
        np.testing.assert_array_equal(P[b][:, :7], ref[:, :7])
        assert (_ulp(P[b][:, 7], ref[:, 7]) <= YAW_ULP).all()
        d = g[f"{name}/dets"][b]
        kept = np.concatenate([np.nonzero((d[:, 9] == j) & (d[:, 0] > np.float32(0.2)))[0]
                               for j in range(3)])
        exact = np.arctan2(d[kept, 7].astype(np.float64), d[kept, 8].astype(np.float64))
        assert (_ulp(P[b][:, 7], exact.astype(np.float32)) <= 1).all()
        # real rows: bit-exact given the kernel's own preds; fixtures up to the yaw column
        split = {j: P[b][R[b][:, 0] == j] for j in range(3)}
        np.testing.assert_array_equal(R[b], po.real_rows(split, 3, "f32"))
        ref_real = g[f"{name}/{b}/real"]
        np.testing.assert_array_equal(R[b][:, :7], ref_real[:, :7])
        assert (_ulp(R[b][:, 7], ref_real[:, 7]) <= YAW_ULP).all()


def test_post_process_numpy1_arith(golden_project, gpu):
    g = golden_project
    dets = torch.from_numpy(g["typical/dets"]).to(gpu)
    preds, real, off = runtime.post_process(dets, arith=_lib.REAL_F64)
    P, R = _split(preds, off), _split(real, off)
    for b in range(dets.shape[0]):
        split = {j: P[b][R[b][:, 0] == j] for j in range(3)}
        np.testing.assert_array_equal(R[b], po.real_rows(split, 3, "f64"))


@pytest.mark.parametrize("name", ["typical", "edges", "e2e"])
def test_project_boxes_matches_reference(golden_project, gpu, name):
    g = golden_project
    names = list(g[f"{name}/calibs"])
    cals, shapes = _calibs(g, names)
    dets = torch.from_numpy(g[f"{name}/dets"]).to(gpu)
    preds, real, off = runtime.post_process(dets)
    boxes, conf, row, ext, boff = runtime.project_boxes(real, off, cals, extents=True)
    Bx, C, Rw, E = (_split(t, boff) for t in (boxes, conf, row, ext))
    Rl = _split(real, off)
    for b in range(dets.shape[0]):
        ob, oc, orow, oext = po.image_boxes(Rl[b], *shapes[b])
        np.testing.assert_array_equal(Bx[b], ob)
        np.testing.assert_array_equal(C[b], oc)
        np.testing.assert_array_equal(Rw[b], orow)
        np.testing.assert_allclose(E[b], oext, rtol=1e-12, atol=1e-9)
        np.testing.assert_array_equal(Bx[b], g[f"{name}/{b}/boxes"])
        np.testing.assert_array_equal(C[b], g[f"{name}/{b}/conf"])


def test_project_score_confidence_and_shared_calib(golden_project, gpu):
    g = golden_project
    cals, shapes = _calibs(g, ["avg"])
    dets = torch.from_numpy(g["e2e/dets"]).to(gpu)
    preds, real, off = runtime.post_process(dets)
    boxes, conf, row, _, boff = runtime.project_boxes(real, off, cals, preds=preds,
                                                      conf_source=_lib.CONF_SCORE)
    P, R = _split(preds, off), _split(real, off)
    ob, oc, orow, _ = po.image_boxes(R[0], *shapes[0], 0.3, P[0][:, 0].astype(np.float64))
    np.testing.assert_array_equal(_split(boxes, boff)[0], ob)
    np.testing.assert_array_equal(_split(conf, boff)[0], oc)
    assert len(ob) > 0


def test_many_frames_random_vs_oracle(gpu):
    """130 frames (> 2 scan chunks, > 16 waves), K = 100 (> one ballot chunk)."""
    import project_cases
    rng = np.random.default_rng(5)
    B, K = 130, 100
    d = np.zeros((B, K, 10), np.float32)
    d[..., 0] = rng.random((B, K))
    d[..., 1:3] = rng.random((B, K, 2)) * 152
    d[..., 3] = 0.8 + rng.random((B, K)) * 1.6
    d[..., 4:7] = [1.2, 0.5, 0.6] + rng.random((B, K, 3)) * [1.0, 2.0, 4.4]
    d[..., 7:9] = rng.random((B, K, 2)) * 2 - 1
    d[..., 9] = rng.integers(0, 4, (B, K))  # class 3 >= num_classes: never kept
    cal_d = project_cases.calibs()
    names = ["avg" if b % 3 else "seq" for b in range(B)]
    cals = [runtime.make_calib(cal_d[n]["V2C"], cal_d[n]["R0"], cal_d[n]["P2"], cal_d[n]["img_shape"])
            for n in names]
    preds, real, off = runtime.post_process(torch.from_numpy(d).to(gpu))
    boxes, conf, row, ext, boff = runtime.project_boxes(real, off, cals, extents=True)
    P, R, Bx, E = _split(preds, off), _split(real, off), _split(boxes, boff), _split(ext, boff)
    n_boxes = 0
    for b in range(B):
        preds_o = po.post_frame(d[b])
        ref = np.concatenate([preds_o[j] for j in range(3)]).reshape(-1, 8)
        np.testing.assert_array_equal(P[b][:, :7], ref[:, :7])
        split = {j: P[b][R[b][:, 0] == j] for j in range(3)}
        real_k = po.real_rows(split, 3, "f32")
        np.testing.assert_array_equal(R[b], real_k)
        ob, oc, orow, oext = po.image_boxes(real_k, cal_d[names[b]], cal_d[names[b]]["img_shape"])
        np.testing.assert_array_equal(Bx[b], ob)
        np.testing.assert_allclose(E[b], oext, rtol=1e-12, atol=1e-9)
        n_boxes += len(ob)
    assert n_boxes > 1000


def test_empty_and_errors(gpu):
    preds, real, off = runtime.post_process(torch.zeros((0, 50, 10), device=gpu))
    assert off.cpu().tolist() == [0]
    preds, real, off = runtime.post_process(torch.zeros((2, 0, 10), device=gpu))
    assert off.cpu().tolist() == [0, 0, 0]
    with pytest.raises(_lib.SfaNativeError):
        runtime.post_process(torch.zeros((1, 5, 10)))  # CPU tensor: no fallback


def test_dropin_convert_sfa3d_to_2d_boxes(golden_project, gpu):
    from utils.fusion_utils import convert_sfa3d_to_2d_boxes

    class Calib:
        pass
    g = golden_project
    for name in ("typical", "edges"):
        for b, cal_name in enumerate(g[f"{name}/calibs"]):
            c = Calib()
            c.V2C, c.R0, c.P2 = (g[f"calib/{cal_name}/{f}"] for f in ("V2C", "R0", "P2"))
            shape = tuple(int(v) for v in g[f"calib/{cal_name}/img_shape"])
            post = {j: g[f"{name}/{b}/post{j}"] for j in range(3)}
            boxes, conf = convert_sfa3d_to_2d_boxes(post, c, shape)
            np.testing.assert_array_equal(np.array(boxes, np.int64).reshape(-1, 4), g[f"{name}/{b}/boxes"])
            np.testing.assert_array_equal(np.array(conf), g[f"{name}/{b}/conf"])
