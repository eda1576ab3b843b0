"""Pin the post-processing / camera-projection oracle against the reference's outputs
(post_processing, convert_det_to_real_values, lidar_to_camera_box,
convert_sfa3d_to_2d_boxes — tests/golden/gen_project_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import project_oracle as po

# numpy's f32 arctan2 is a SIMD approximation (up to 3 ulp off the correctly rounded
# value on AVX-512 hosts): yaw is compared within 4 ulp, everything else exactly.
YAW_ULP = 4


def _ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


def frames(g):
    for name in ("typical", "edges", "e2e"):
        dets = g[f"{name}/dets"]
        for b, cal in enumerate(g[f"{name}/calibs"]):
            yield name, b, dets[b], str(cal)


def calib(g, n):
    return {f: g[f"calib/{n}/{f}"] for f in ("V2C", "R0", "P2")}, tuple(g[f"calib/{n}/img_shape"])


def test_post_frame_matches_reference(golden_project):
    g = golden_project
    for name, b, det, _ in frames(g):
        post = po.post_frame(det)
        for j in range(3):
            ref = g[f"{name}/{b}/post{j}"]
            assert post[j].dtype == np.float32 and post[j].shape == ref.shape, (name, b, j)
            np.testing.assert_array_equal(post[j][:, :7], ref[:, :7])
            assert (_ulp_diff(post[j][:, 7], ref[:, 7]) <= YAW_ULP).all()


def test_real_rows_match_reference(golden_project):
    g = golden_project
    for name, b, _, _ in frames(g):
        post = {j: g[f"{name}/{b}/post{j}"] for j in range(3)}
        np.testing.assert_array_equal(po.real_rows(post, 3, "f32"), g[f"{name}/{b}/real"])
        # numpy 1.x (f64) variant: same rows within f32 rounding of metres
        r64 = po.real_rows(post, 3, "f64")
        np.testing.assert_allclose(r64, g[f"{name}/{b}/real"], rtol=2e-7, atol=1e-5)


def test_camera_boxes_match_reference(golden_project):
    g = golden_project
    for name, b, _, cal in frames(g):
        c, _ = calib(g, cal)
        real = g[f"{name}/{b}/real"]
        cam = np.array([po.lidar_to_camera(r[1:], c["V2C"], c["R0"]) for r in real]).reshape(-1, 7)
        np.testing.assert_allclose(cam, g[f"{name}/{b}/cam"], rtol=1e-13, atol=1e-12)


def test_image_boxes_match_reference(golden_project):
    g = golden_project
    total = 0
    for name, b, _, cal in frames(g):
        c, shape = calib(g, cal)
        boxes, conf, rows, ext = po.image_boxes(g[f"{name}/{b}/real"], c, shape)
        np.testing.assert_array_equal(boxes, g[f"{name}/{b}/boxes"])
        np.testing.assert_array_equal(conf, g[f"{name}/{b}/conf"])
        assert (ext[:, 2] > ext[:, 0]).all() and (ext[:, 3] > ext[:, 1]).all()
        total += len(boxes)
    assert total > 50  # the fixtures exercise the projection


def test_score_confidence_variant_keeps_class0():
    det = np.zeros((3, 10), np.float32)
    det[:, 0] = [0.9, 0.5, 0.25]
    det[:, 2] = 60  # 19.7 m ahead
    det[:, 1] = 76
    det[:, 3:7] = [1.5, 1.5, 1.6, 3.9]
    det[:, 8] = 1
    det[:, 9] = [0, 1, 2]
    post = po.post_frame(det)
    real = po.real_rows(post)
    cal = {"V2C": np.eye(3, 4)[[1, 2, 0]] * [[-1], [-1], [1]], "R0": np.eye(3),
           "P2": np.array([[700, 0, 600, 0], [0, 700, 180, 0], [0, 0, 1, 0]], float)}
    b_cls = po.image_boxes(real, cal, (375, 1242))
    sc = np.concatenate([post[j][:, 0] for j in range(3)]).astype(np.float64)
    b_sc = po.image_boxes(real, cal, (375, 1242), 0.3, sc)
    assert list(b_cls[1]) == [1.0, 2.0]                 # class ids; class 0 dropped
    assert np.allclose(b_sc[1], [0.9, 0.5])              # scores; 0.25 < 0.3 dropped
