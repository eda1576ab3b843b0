#!/usr/bin/env python3
"""Golden fixtures for the back view of demo_2_sides.py, made by running
the REFERENCE in the build container (same import recipe as gen_golden.py):

  data_process/demo_dataset.py:70-88   back map = makeBEVMap(get_filtered_lidar(sweep,
                                       boundary_back), boundary_back) — rows come from
                                       floor(x / D) with x < 0: numpy wraps the negative
                                       indices (kitti_bev_utils.py:28, 44-48)
  utils/demo_utils.py:109-127          do_detect(..., is_front=False): torch.flip(bevmap,
                                       [1, 2]) -> model -> _sigmoid -> decode -> post_processing

on the synthetic sweep of seed 1 (also the e2e model fixture's sweep) with the fixture weights
(seed 0).  Output: tests/golden/back_golden.npz.
"""

from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as gg  # noqa: E402

BACK = {"minX": -50, "maxX": 0, "minY": -25, "maxY": 25, "minZ": -2.73, "maxZ": 1.27}


def main():
    import torch
    if not os.path.isdir(gg.REF):
        sys.exit("reference not present")
    ref = gg._import_reference()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    res = {}
    for seed in (1, 3):
        cloud = gg.synthetic.synthetic_point_cloud(seed)
        filt = ref["data"].get_filtered_lidar(cloud.copy(), BACK)
        bev = ref["bev"].makeBEVMap(filt, BACK)
        flat = bev.reshape(3, -1)
        nz = np.nonzero(np.any(flat != 0, axis=0))[0].astype(np.int32)
        k = f"s{seed}"
        res[f"{k}/filtered_n"] = np.array(filt.shape[0])
        res[f"{k}/cells"] = nz
        res[f"{k}/intensity"] = flat[0, nz]
        res[f"{k}/height"] = flat[1, nz]
        res[f"{k}/density"] = flat[2, nz]
        res[f"{k}/map_sha"] = np.array(gg._sha(bev))
        print(f"back {k}: kept {filt.shape[0]}, cells {nz.size}")
    # do_detect on the back view of seed 1
    model, _ = gg._ref_model(ref, seed=0)
    cloud = gg.synthetic.synthetic_point_cloud(1)
    bev = ref["bev"].makeBEVMap(ref["data"].get_filtered_lidar(cloud.copy(), BACK), BACK)
    with torch.no_grad():
        x = torch.flip(torch.from_numpy(bev), [1, 2]).unsqueeze(0).float()
        outs = model(x)
        for h in gg.HEADS:
            res[f"detect/{h}"] = outs[h].numpy().copy()
        hm = ref["tu"]._sigmoid(outs["hm_cen"])
        off = ref["tu"]._sigmoid(outs["cen_offset"])
        dets = ref["ev"].decode(hm, off, outs["direction"], outs["z_coor"], outs["dim"], K=50).numpy()
    post = gg._quiet(ref["ev"].post_processing, dets.copy(), 3, 4, 0.2)
    res["detect/dets"] = dets
    for j in range(3):
        res[f"detect/post{j}"] = post[0][j]
    print(f"back detect: dets {dets.shape}, post {[post[0][j].shape[0] for j in range(3)]}")
    np.savez_compressed(os.path.join(HERE, "back_golden.npz"), **res)


if __name__ == "__main__":
    main()
