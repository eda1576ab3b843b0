"""The reference callers' DataLoader loop through the drop-in, on the GPU:
HIP is initialised first (the model is created on the GPU, test.py:106-112), then the drop-in
create_test_dataloader runs with num_workers = 1 (test.py:39,120) over a synthetic KITTI tree.
The workers only read the .bin files; the batch's maps are made on the GPU in the main process:
  * bev_maps are (B, 3, 608, 608) float64 CPU tensors bit-exact with the oracle's
    makeBEVMap(get_filtered_lidar(sweep)) (ragged last batch, an empty sweep);
  * the callers' sequence on them — .to(device).float() (test.py:124), model (:133), _sigmoid
    (:150, :167), decode K = 50 (:170) — gives the detections of the resident pipeline
    (DetectorPipeline: raw sweeps -> BEV -> forward -> decode on the device), bit for bit."""
import numpy as np
import pytest
import torch

import golden_cases as gc
import loader_cases as lc
from oracle import bev_oracle
from sfa_hip import runtime

pytestmark = pytest.mark.gpu


def test_test_loader_loop_like_test_py(tmp_path, gpu, golden, monkeypatch):
    from data_process.kitti_dataloader import create_test_dataloader
    from data_process.kitti_dataset import KittiDataset
    from models.model_utils import create_model
    from utils.evaluation_utils import decode
    from utils.torch_utils import _sigmoid
    monkeypatch.setattr(KittiDataset, "get_image", lc.stub_image)
    ids, clouds = lc.make_tree(str(tmp_path))
    cfg = lc.Cfg(arch="fpn_resnet_18", heads=dict(gc.HEADS), head_conv=64, imagenet_pretrained=False)
    model = create_model(cfg)
    sd = gc.state_dict_np(golden.model)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model = model.to(gpu).eval()
    torch.cuda.synchronize()  # HIP is up before the workers fork
    loader = create_test_dataloader(lc.configs(str(tmp_path), batch_size=2, num_workers=1))
    pipe = runtime.DetectorPipeline(model._engine(gpu), 2, K=50, with_bev=True,
                                    max_points=max(1, sum(c.shape[0] for c in clouds.values())))
    seen = []
    for metadatas, bev_maps, img_rgbs in loader:
        sids = [int(p[-10:-4]) for p in metadatas["img_path"]]
        seen += sids
        assert bev_maps.dtype == torch.float64 and bev_maps.device.type == "cpu"
        assert tuple(bev_maps.shape) == (len(sids), 3, 608, 608)
        for i, sid in enumerate(sids):
            exp = bev_oracle.makeBEVMap(bev_oracle.get_filtered_lidar(clouds[sid], gc.BOUNDARY), gc.BOUNDARY)
            np.testing.assert_array_equal(bev_maps[i].numpy(), exp, err_msg=f"sample {sid}")
        with torch.no_grad():
            outputs = model(bev_maps.to(gpu).float())
            outputs["hm_cen"] = _sigmoid(outputs["hm_cen"])
            outputs["cen_offset"] = _sigmoid(outputs["cen_offset"])
            dets = decode(outputs["hm_cen"], outputs["cen_offset"], outputs["direction"], outputs["z_coor"],
                          outputs["dim"], K=50).cpu().numpy()
        cl = [clouds[s] for s in sids] + [np.zeros((0, 4), np.float32)] * (2 - len(sids))
        pipe.set_points(cl)
        ref = pipe.run().cpu().numpy()[:len(sids)]
        np.testing.assert_array_equal(dets, ref)
    assert seen == ids


def test_test_loader_bev_on_device(tmp_path, gpu, golden, monkeypatch):
    """Opt-in configs.bev_on_device: the loader yields the (B, 3, 608, 608) maps
    as float32 tensors already on the GPU (no f64 device-to-host copy and back). They equal the
    default mode's f64 CPU maps cast to float32 (what test.py:124 makes of them), and the callers'
    .to(device).float() -> model -> _sigmoid -> decode sequence gives bit-equal detections in both
    modes; the default stays the reference's f64 CPU tensor."""
    from data_process.kitti_dataloader import create_test_dataloader
    from data_process.kitti_dataset import KittiDataset
    from models.model_utils import create_model
    from utils.evaluation_utils import decode
    from utils.torch_utils import _sigmoid
    monkeypatch.setattr(KittiDataset, "get_image", lc.stub_image)
    ids, clouds = lc.make_tree(str(tmp_path))
    cfg = lc.Cfg(arch="fpn_resnet_18", heads=dict(gc.HEADS), head_conv=64, imagenet_pretrained=False)
    model = create_model(cfg)
    sd = gc.state_dict_np(golden.model)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model = model.to(gpu).eval()
    torch.cuda.synchronize()

    def run(on_device):
        conf = lc.configs(str(tmp_path), batch_size=2, num_workers=1)
        if on_device is not None:
            conf.bev_on_device = on_device
            conf.device = gpu
        maps, dets = [], []
        for _, bev_maps, _ in create_test_dataloader(conf):
            if on_device:
                assert bev_maps.dtype == torch.float32 and bev_maps.device == gpu
            else:
                assert bev_maps.dtype == torch.float64 and bev_maps.device.type == "cpu"
            maps.append(bev_maps.cpu())
            with torch.no_grad():
                out = model(bev_maps.to(gpu).float())
                out["hm_cen"] = _sigmoid(out["hm_cen"])
                out["cen_offset"] = _sigmoid(out["cen_offset"])
                dets.append(decode(out["hm_cen"], out["cen_offset"], out["direction"], out["z_coor"], out["dim"],
                                   K=50).cpu().numpy())
        return maps, dets

    m_host, d_host = run(None)
    m_off, d_off = run(False)
    m_dev, d_dev = run(True)
    assert len(m_host) == len(m_dev) == len(m_off) == (len(ids) + 1) // 2
    for a, b, c in zip(m_host, m_off, m_dev):
        np.testing.assert_array_equal(a.numpy(), b.numpy())
        np.testing.assert_array_equal(a.float().numpy(), c.numpy())
    for a, b, c in zip(d_host, d_off, d_dev):
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(a, c)


def test_deferred_bev_train_hflip(gpu):
    """The train-mode deferred BEV (kitti_dataset.py:93-97: hflipped maps): a batch of
    DeferredBEV sweeps with and without flip_w, voxelised by DeferredBEVBatch in both output modes,
    equals the oracle's makeBEVMap(get_filtered_lidar(sweep)) flipped on the last axis where flip_w is
    set (bit-exact in f64; the on-device float32 maps are those values rounded)."""
    from data_process.kitti_dataloader import DeferredBEVBatch
    from data_process.kitti_dataset import DeferredBEV
    from sfa_hip import synthetic as syn
    clouds = [syn.synthetic_point_cloud(300 + j)[:: 1 + j].copy() for j in range(3)]
    flips = [True, False, True]
    batch = DeferredBEVBatch([DeferredBEV(c, f) for c, f in zip(clouds, flips)])
    host = batch.voxelize(gpu)
    dev = batch.voxelize(gpu, on_device=True)
    assert host.dtype == torch.float64 and host.device.type == "cpu"
    assert dev.dtype == torch.float32 and dev.device == gpu
    for i, (c, f) in enumerate(zip(clouds, flips)):
        exp = bev_oracle.makeBEVMap(bev_oracle.get_filtered_lidar(c, gc.BOUNDARY), gc.BOUNDARY)
        if f:
            exp = exp[..., ::-1]
        np.testing.assert_array_equal(host[i].numpy(), exp, err_msg=f"sweep {i} (flip {f})")
        np.testing.assert_array_equal(dev[i].cpu().numpy(), exp.astype(np.float32), err_msg=f"sweep {i} on device")
