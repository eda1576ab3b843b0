"""Pin the fusion oracle against the reference fusion functions' outputs (CPU)."""
import numpy as np
import pytest

import fusion_cases
from oracle import fusion_oracle as fo

CASES = list(fusion_cases.cases())


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("mode,tag", [("bayes", "bayes"), ("weighted", "weighted")])
def test_fusion_oracle_matches_reference(golden_fusion, name, mode, tag):
    g = golden_fusion
    case = fusion_cases.cases()[name]
    fused, keep = fo.run(case, mode)
    np.testing.assert_array_equal(np.array([f[0] for f in fused], np.int64).reshape(-1, 4),
                                  g[f"{name}/{tag}/box"])
    np.testing.assert_array_equal(np.array([f[1] for f in fused]), g[f"{name}/{tag}/conf"])
    np.testing.assert_array_equal(np.array([f[2] for f in fused], np.int64), g[f"{name}/{tag}/cls"])
    np.testing.assert_array_equal(np.array([f[3] for f in fused], np.int64), g[f"{name}/{tag}/src"])
    kept = [fused[i] for i in keep]
    np.testing.assert_array_equal(np.array([f[0] for f in kept], np.int64).reshape(-1, 4),
                                  g[f"{name}/{tag}_nms/box"])
    np.testing.assert_array_equal(np.array([f[1] for f in kept]), g[f"{name}/{tag}_nms/conf"])


@pytest.mark.parametrize("name", CASES)
def test_iou_matrix(golden_fusion, name):
    case = fusion_cases.cases()[name]
    m = np.array([[fo.iou(a, b) for b in case["sfa_boxes"]] for a in case["yolo_boxes"]],
                 np.float64).reshape(len(case["yolo_boxes"]), len(case["sfa_boxes"]))
    np.testing.assert_array_equal(m, golden_fusion[f"{name}/iou"])


def test_gaussian_nms_oracle_matches_readme_snippet(golden_gaussian_nms):
    """oracle.gaussian_nms == the README's gaussian_nms (README.md:250-261) as run by
    tests/golden/gen_gaussian_nms_golden.py, bit for bit (same numpy exp)."""
    from conftest import gaussian_nms_case_names
    g = golden_gaussian_nms
    names = gaussian_nms_case_names(g)
    assert len(names) >= 9
    for name in names:
        got = fo.gaussian_nms(g[f"{name}/boxes"].tolist(), g[f"{name}/conf_in"], float(g[f"{name}/sigma"]))
        np.testing.assert_array_equal(np.array(got, np.float64), g[f"{name}/conf_out"], err_msg=name)
