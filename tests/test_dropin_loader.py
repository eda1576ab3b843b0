"""The drop-in DataLoader: its workers only read files — every sample's BEV
map is deferred to the main process (data_process.kitti_dataloader), so a caller that initialised
HIP before creating the loader (test.py:112 then :120, --num_workers 1) works; a HIP host API
called in a worker forked after HIP init raises a clear SfaNativeError.  CPU-only checks here (no
HIP: the worker path must not need it); tests/test_gpu_dropin_loader.py runs the whole loop on the GPU."""
import numpy as np
import pytest
import torch

import loader_cases as lc
from sfa_hip import _lib


def _no_hip(*a, **k):
    raise AssertionError("HIP used where it must not be (a DataLoader worker)")


def test_workers_only_read_files(tmp_path, monkeypatch):
    from data_process import kitti_dataloader as kdl
    from data_process.kitti_dataset import KittiDataset
    monkeypatch.setattr(KittiDataset, "get_image", lc.stub_image)
    ids, clouds = lc.make_tree(str(tmp_path))
    monkeypatch.setattr(_lib, "lib", _no_hip)  # inherited by the forked worker
    loader = kdl.create_test_dataloader(lc.configs(str(tmp_path), batch_size=2, num_workers=1))
    assert len(loader) == 3 and loader.batch_size == 2 and loader.dataset.defer_bev
    seen = []
    for metadatas, bev, img in loader.loader:  # the worker's batches, before the main process resolves them
        assert isinstance(bev, kdl.DeferredBEVBatch)
        assert isinstance(img, torch.Tensor) and img.dtype == torch.uint8
        for p, d in zip(metadatas["img_path"], bev.items):
            sid = int(p[-10:-4])
            np.testing.assert_array_equal(d.points, clouds[sid])  # == np.fromfile(...).reshape(-1, 4)
            assert not d.flip_w
            seen.append(sid)
    assert seen == ids


def test_bev_in_a_forked_worker_raises_clearly(monkeypatch):
    from data_process.kitti_bev_utils import makeBEVMap
    from data_process.kitti_data_utils import get_filtered_lidar
    monkeypatch.setattr(torch.cuda, "_is_in_bad_fork", lambda: True)
    for fn, args in ((makeBEVMap, (np.zeros((3, 4), np.float32), {})), (get_filtered_lidar, (np.zeros((3, 4), np.float32), {}))):
        with pytest.raises(_lib.SfaNativeError, match="forked after HIP was initialised"):
            fn(*args)


def test_collate_keeps_other_fields():
    from data_process import kitti_dataloader as kdl
    from data_process.kitti_dataset import DeferredBEV
    batch = [({"img_path": "a"}, DeferredBEV(np.ones((2, 4), np.float32)), np.zeros((2, 2), np.uint8)),
             ({"img_path": "b"}, DeferredBEV(np.zeros((0, 4), np.float32), True), np.ones((2, 2), np.uint8))]
    meta, bev, img = kdl.bev_collate(batch)
    assert meta == {"img_path": ["a", "b"]}
    assert isinstance(bev, kdl.DeferredBEVBatch) and [d.flip_w for d in bev.items] == [False, True]
    assert img.shape == (2, 2, 2)


def test_bev_on_device_with_cpu_device_refused(tmp_path, monkeypatch):
    """configs.bev_on_device with a CPU configs.device is refused up front (no silent GPU choice)."""
    from data_process import kitti_dataloader as kdl
    from data_process.kitti_dataset import KittiDataset
    monkeypatch.setattr(KittiDataset, "get_image", lc.stub_image)
    lc.make_tree(str(tmp_path))
    cfg = lc.configs(str(tmp_path), batch_size=2, num_workers=0)
    cfg["bev_on_device"] = True
    cfg["device"] = torch.device("cpu")
    with pytest.raises(ValueError, match="bev_on_device needs a CUDA"):
        kdl.create_test_dataloader(cfg)
    cfg["bev_on_device"] = False  # the reference's CPU maps: still fine with a CPU device
    assert len(kdl.create_test_dataloader(cfg)) == 3
