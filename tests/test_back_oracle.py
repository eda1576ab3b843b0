"""Pin the oracle on the back view of demo_2_sides.py (tests/golden/gen_back_golden.py: the
reference's boundary_back map, and do_detect's flip -> forward -> decode on it).  CPU only."""
import hashlib

import numpy as np
import pytest
import torch

import golden_cases as gc
from oracle import bev_oracle, decode_oracle, model_oracle
from sfa_hip import synthetic

BACK = {"minX": -50, "maxX": 0, "minY": -25, "maxY": 25, "minZ": -2.73, "maxZ": 1.27}


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("seed", [1, 3])
def test_back_bev_oracle_matches_reference(golden_back, seed):
    g, k = golden_back, f"s{seed}"
    filt = bev_oracle.get_filtered_lidar(synthetic.synthetic_point_cloud(seed), BACK)
    assert filt.shape[0] == int(g[f"{k}/filtered_n"])
    bev = bev_oracle.makeBEVMap(filt, BACK)
    assert _sha(bev) == str(g[f"{k}/map_sha"])
    flat = bev.reshape(3, -1)
    np.testing.assert_array_equal(flat[0, g[f"{k}/cells"]], g[f"{k}/intensity"])
    np.testing.assert_array_equal(flat[2, g[f"{k}/cells"]], g[f"{k}/density"])


def test_back_detect_oracle_matches_reference(golden_back, golden):
    g = golden_back
    bev = bev_oracle.makeBEVMap(
        bev_oracle.get_filtered_lidar(synthetic.synthetic_point_cloud(1), BACK), BACK)
    torch.set_num_threads(8)
    sd = model_oracle.state_dict_torch(gc.state_dict_np(golden.model))
    x = torch.from_numpy(np.ascontiguousarray(bev[:, ::-1, ::-1])).unsqueeze(0).float()
    with torch.no_grad():
        out = model_oracle.forward(sd, x)
    for h in gc.HEADS:
        ref = g[f"detect/{h}"]
        assert np.max(np.abs(out[h].numpy() - ref) / np.maximum(1, np.abs(ref))) <= 1e-5
    # decode on the reference's own logits: the oracle decode is exact
    hm = decode_oracle.sigmoid_clamp(g["detect/hm_cen"])
    off = decode_oracle.sigmoid_clamp(g["detect/cen_offset"])
    dets = decode_oracle.decode(hm, off, g["detect/direction"], g["detect/z_coor"], g["detect/dim"],
                                K=50)
    np.testing.assert_array_equal(dets, g["detect/dets"])
