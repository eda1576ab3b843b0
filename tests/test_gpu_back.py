"""GPU parity of the back view (demo_2_sides.py): boundary_back voxelisation
with the flip fused (SFA_BEV_FLIP_HW), the flipped model input (SFA_IN_NCHW3_FLIP_HW), the
do_detect drop-in, and the two-sided pipeline — against the reference-generated back fixtures.

Tolerances: BEV maps bit-exact; logits 1e-4 * max(1, |ref|) (as tests/test_gpu_model.py);
flip-fused paths bit-exact against the same kernels on explicitly flipped inputs."""
import hashlib

import numpy as np
import pytest
import torch

import golden_cases as gc
from sfa_hip import _lib, runtime, synthetic

pytestmark = pytest.mark.gpu
TOL = 1e-4
BACK = runtime.DEFAULT_BOUNDARY_BACK


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


class Cfg(dict):
    __getattr__ = dict.__getitem__


def _model(golden, dev):
    from models.model_utils import create_model
    m = create_model(Cfg(arch="fpn_resnet_18", heads=dict(gc.HEADS), head_conv=64,
                         imagenet_pretrained=False))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in gc.state_dict_np(golden.model).items()})
    return m.to(dev).eval()


@pytest.mark.parametrize("seed", [1, 3])
def test_back_bev_flip_bit_exact(golden_back, gpu, seed):
    cloud = torch.from_numpy(synthetic.synthetic_point_cloud(seed)).to(gpu)
    vox = runtime.BevVoxelizer(gpu, 1)
    plain = vox(cloud, [0, cloud.shape[0]], BACK, _lib.BEV_NCHW3_F64, _lib.BEV_RAW).cpu().numpy()[0]
    assert _sha(plain) == str(golden_back[f"s{seed}/map_sha"])
    flip = vox(cloud, [0, cloud.shape[0]], BACK, _lib.BEV_NCHW3_F64,
               _lib.BEV_RAW | _lib.BEV_FLIP_HW).cpu().numpy()[0]
    np.testing.assert_array_equal(flip, plain[:, ::-1, ::-1])
    n4 = vox(cloud, [0, cloud.shape[0]], BACK, _lib.BEV_NHWC4_F32, _lib.BEV_RAW | _lib.BEV_FLIP_HW)
    np.testing.assert_array_equal(n4.cpu().numpy()[0, ..., :3],
                                  plain[:, ::-1, ::-1].transpose(1, 2, 0).astype(np.float32))


def test_flipped_input_layout(golden, golden_back, gpu):
    model = _model(golden, gpu)
    bev = torch.from_numpy(synthetic.synthetic_bev(2, 160, 192, seed=7)).to(gpu)
    with torch.no_grad():
        a = model.forward_layout(bev, _lib.IN_NCHW3_FLIP_HW)
        b = model(torch.flip(bev, [2, 3]).contiguous())
    for h in gc.HEADS:
        np.testing.assert_array_equal(a[h].cpu().numpy(), b[h].cpu().numpy())


def test_do_detect_back_matches_reference(golden, golden_back, gpu):
    from data_process.kitti_bev_utils import makeBEVMap
    from data_process.kitti_data_utils import get_filtered_lidar
    from utils.demo_utils import do_detect
    model = _model(golden, gpu)
    cloud = synthetic.synthetic_point_cloud(1)
    bevmap = torch.from_numpy(makeBEVMap(get_filtered_lidar(cloud, BACK), BACK))
    cfg = Cfg(device=gpu, K=50, num_classes=3, down_ratio=4, peak_thresh=0.2)
    dets, shown, fps = do_detect(cfg, model, bevmap, is_front=False)
    np.testing.assert_array_equal(shown.numpy(), torch.flip(bevmap, [1, 2]).numpy())
    # logits of the flipped map vs the reference's
    x = bevmap.unsqueeze(0).to(gpu).float()
    with torch.no_grad():
        out = model.forward_layout(x, _lib.IN_NCHW3_FLIP_HW)
    for h in gc.HEADS:
        ref = golden_back[f"detect/{h}"]
        e = float(np.max(np.abs(out[h].cpu().numpy() - ref) / np.maximum(1, np.abs(ref))))
        print(f"back {h}: max rel err {e:.3g}")
        assert e <= TOL
    ref_post = [golden_back[f"detect/post{j}"] for j in range(3)]
    for j in range(3):
        assert abs(len(dets[j]) - len(ref_post[j])) <= 1
    # scores (sorted) within tolerance; identities where the reference's gaps are unambiguous
    got = np.sort(dets[0][:, 0])[::-1]
    ref = np.sort(ref_post[0][:, 0])[::-1]
    n = min(len(got), len(ref))
    assert np.max(np.abs(got[:n] - ref[:n])) <= TOL
    assert fps > 0


def test_two_sided_pipeline_matches_separate_views(golden, gpu):
    arch = _lib.make_arch(gc.HEADS)
    eng = runtime.KfpnEngine(arch, runtime.pack_state_dict(gc.state_dict_np(golden.model), arch), gpu)
    clouds = [synthetic.synthetic_point_cloud(s) for s in (1, 2)]
    pipe = runtime.DetectorPipeline(eng, 2, K=50, with_bev=True, two_sided=True,
                                    max_points=sum(c.shape[0] for c in clouds))
    pipe.set_points(clouds)
    dets = pipe.run().cpu().numpy()
    vox = runtime.BevVoxelizer(gpu, 2)
    pts = torch.from_numpy(np.concatenate(clouds)).to(gpu)
    offs = [0, clouds[0].shape[0], clouds[0].shape[0] + clouds[1].shape[0]]
    back = vox(pts, offs, BACK, _lib.BEV_NCHW3_F32, _lib.BEV_RAW)
    outs = eng.forward(back, _lib.IN_NCHW3_FLIP_HW)
    ref = runtime.decode(outs["hm_cen"], outs["cen_offset"], outs["direction"], outs["z_coor"],
                         outs["dim"], K=50, apply_sigmoid=True).cpu().numpy()
    np.testing.assert_array_equal(dets[2:], ref)
    front = vox(pts, offs, runtime.DEFAULT_BOUNDARY, _lib.BEV_NCHW3_F32, _lib.BEV_RAW)
    outs = eng.forward(front)
    ref = runtime.decode(outs["hm_cen"], outs["cen_offset"], outs["direction"], outs["z_coor"],
                         outs["dim"], K=50, apply_sigmoid=True).cpu().numpy()
    np.testing.assert_array_equal(dets[:2], ref)
