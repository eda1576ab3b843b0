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
