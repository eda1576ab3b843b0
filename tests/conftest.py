import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SFA_ROOT = os.path.join(REPO, "lidar-image_object-detection_-fpn_resnet-yolov8_amd", "sfa")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, SFA_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    class G:
        bev = np.load(os.path.join(GOLDEN, "bev_golden.npz"))
        decode = np.load(os.path.join(GOLDEN, "decode_golden.npz"))
        model = np.load(os.path.join(GOLDEN, "model_golden.npz"))
    return G


@pytest.fixture(scope="session")
def golden_bench():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "bench_golden.npz"))


@pytest.fixture(scope="session")
def golden_fusion():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "fusion_golden.npz"))


@pytest.fixture(scope="session")
def golden_gaussian_nms():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "gaussian_nms_golden.npz"))


def gaussian_nms_case_names(g):
    return sorted({k.split("/")[0] for k in g.files})


@pytest.fixture(scope="session")
def golden_back():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "back_golden.npz"))


@pytest.fixture(scope="session")
def golden_project():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "project_golden.npz"))


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.skip("no GPU visible")
    import torch
    return torch.device("cuda", 0)


def pytest_collection_modifyitems(config, items):
    # GPU tests must never silently pass on a CPU box: they are skipped here and
    # run on the MI355X with `-m gpu`.
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible (run with -m gpu on an MI355X)")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
