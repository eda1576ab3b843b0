"""A synthetic KITTI tree for the drop-in DataLoader tests: testing/velodyne/NNNNNN.bin
(synthetic sweeps, one empty, one subsampled), ImageSets/test.txt, and a reference-style
`configs` object (test.py:31-79 fields the loader reads)."""
import os

import numpy as np

from sfa_hip import synthetic


class Cfg(dict):
    __getattr__ = dict.__getitem__

    def __setattr__(self, k, v):
        self[k] = v


def make_tree(root, n=5):
    vel = os.path.join(root, "testing", "velodyne")
    os.makedirs(vel, exist_ok=True)
    os.makedirs(os.path.join(root, "ImageSets"), exist_ok=True)
    ids = list(range(3, 3 + n))
    clouds = {}
    for j, sid in enumerate(ids):
        c = synthetic.synthetic_point_cloud(200 + j)
        if j == 1:
            c = c[::5].copy()
        if j == 3:
            c = np.zeros((0, 4), np.float32)
        c.tofile(os.path.join(vel, f"{sid:06d}.bin"))
        clouds[sid] = c
    with open(os.path.join(root, "ImageSets", "test.txt"), "w") as f:
        f.write("\n".join(str(i) for i in ids) + "\n")
    return ids, clouds


def configs(root, batch_size=2, num_workers=1):
    return Cfg(dataset_dir=root, input_size=(608, 608), hm_size=(152, 152), num_classes=3, max_objects=50,
               num_samples=None, batch_size=batch_size, num_workers=num_workers, pin_memory=False,
               distributed=False)


def stub_image(self, idx):
    """KittiDataset.get_image without cv2 / image files: a small deterministic RGB array."""
    img = np.full((4, 6, 3), idx % 251, np.uint8)
    return os.path.join(self.image_dir, f"{idx:06d}.png"), img
