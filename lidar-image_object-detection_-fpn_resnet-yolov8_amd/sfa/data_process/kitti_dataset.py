"""Drop-in for the reference's data_process/kitti_dataset.py: a KittiDataset whose DataLoader
workers never touch HIP.

The reference runs get_filtered_lidar + makeBEVMap inside ``__getitem__``
(``kitti_dataset.py:60-73`` test mode, ``:75-106`` train / val), i.e. in the DataLoader's worker
processes (``test.py:39,120``: ``--num_workers`` 1).  Its callers create the model on the GPU first
(``test.py:112``), so a worker is a process forked after HIP was initialised and cannot use the GPU
(torch raises "Cannot re-initialize CUDA in forked subprocess").  Here, when the dataset serves a
drop-in loader (``data_process.kitti_dataloader``, which sets ``defer_bev``), a sample carries its
raw sweep as a :class:`DeferredBEV` — the worker only reads files — and the loader voxelises each
batch on the GPU in the main process (one ``sfa_bev_voxelize`` call, filter fused) before the
caller sees it: the same ``(metadatas, bev_maps, img_rgbs)`` batches, bev_maps the (B, 3, 608, 608)
float64 CPU tensor the reference's collate produces (bit-exact maps).  Used directly
(``dataset[i]`` in the main process, no loader) a sample is built eagerly, as in the reference.

Restated from the reference (file I/O, :24-73, :108-122): the constructor's paths and sample list,
``load_img_only``, ``get_image``, ``get_lidar``, ``get_calib``; ``load_img_with_targets`` (:75-106)
keeps the reference's order of label transform, augmentation, filtering, flip draw and targets,
with the point filter and the map deferred like test mode.  The training helpers (``get_label``,
``build_targets``, ``draw_img_with_label``) come from the reference module itself (methods this
class does not define are looked up on the reference's KittiDataset), so a reference tree on
``sys.path`` is needed only for train / val mode.
"""

from __future__ import annotations

import os

import numpy as np
import torch
from torch.utils.data import Dataset

import config.kitti_config as cnf
from sfa_hip import dropin as _dropin


class DeferredBEV:
    """A sample's BEV map, still to be made: its raw (N, 4) float32 sweep (the points the
    reference would pass to get_filtered_lidar), and whether the map is flipped on W afterwards
    (train-mode hflip, kitti_dataset.py:93-97).  Resolved per batch by
    ``data_process.kitti_dataloader`` in the main process."""

    __slots__ = ("points", "flip_w")

    def __init__(self, points: np.ndarray, flip_w: bool = False):
        self.points = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 4)
        self.flip_w = bool(flip_w)

    def __reduce__(self):  # workers pickle samples to the main process
        return DeferredBEV, (self.points, self.flip_w)


def _reference_class():
    ref = _dropin.reference_module("data_process.kitti_dataset")
    if ref is None:
        raise AttributeError("the reference's data_process/kitti_dataset.py (training helpers) is not "
                             "reachable: put the reference's sfa dir on sys.path or set SFA_REFERENCE_ROOT")
    return ref.KittiDataset


class KittiDataset(Dataset):
    def __init__(self, configs, mode="train", lidar_aug=None, hflip_prob=None, num_samples=None):
        self.dataset_dir = configs.dataset_dir
        self.input_size = configs.input_size
        self.hm_size = configs.hm_size
        self.num_classes = configs.num_classes
        self.max_objects = configs.max_objects
        assert mode in ["train", "val", "test"], "Invalid mode: {}".format(mode)
        self.mode = mode
        self.is_test = self.mode == "test"
        sub_folder = "testing" if self.is_test else "training"
        self.lidar_aug = lidar_aug
        self.hflip_prob = hflip_prob
        self.image_dir = os.path.join(self.dataset_dir, sub_folder, "image_2")
        self.lidar_dir = os.path.join(self.dataset_dir, sub_folder, "velodyne")
        self.calib_dir = os.path.join(self.dataset_dir, sub_folder, "calib")
        self.label_dir = os.path.join(self.dataset_dir, sub_folder, "label_2")
        split_txt_path = os.path.join(self.dataset_dir, "ImageSets", "{}.txt".format(mode))
        with open(split_txt_path) as f:
            self.sample_id_list = [int(x.strip()) for x in f.readlines()]
        if num_samples is not None:
            self.sample_id_list = self.sample_id_list[:num_samples]
        self.num_samples = len(self.sample_id_list)
        # set by the drop-in loaders: samples carry DeferredBEV, the loader makes the maps per batch
        self.defer_bev = False

    def __len__(self):
        return len(self.sample_id_list)

    def __getitem__(self, index):
        if self.is_test:
            return self.load_img_only(index)
        return self.load_img_with_targets(index)

    def _bev(self, lidar, flip_w=False):
        if self.defer_bev:
            return DeferredBEV(lidar, flip_w)
        from data_process.kitti_bev_utils import makeBEVMap
        from data_process.kitti_data_utils import get_filtered_lidar
        bev = torch.from_numpy(makeBEVMap(get_filtered_lidar(lidar, cnf.boundary), cnf.boundary))
        return torch.flip(bev, [-1]) if flip_w else bev

    def load_img_only(self, index):
        """Test mode (:60-73): metadatas, the BEV map (or its DeferredBEV), the RGB image."""
        sample_id = int(self.sample_id_list[index])
        img_path, img_rgb = self.get_image(sample_id)
        lidar = self.get_lidar(sample_id)
        return {"img_path": img_path}, self._bev(lidar), img_rgb

    def load_img_with_targets(self, index):
        """Train / val mode (:75-106), the map deferred like test mode."""
        from data_process import transformation
        from data_process.kitti_data_utils import filter_labels
        sample_id = int(self.sample_id_list[index])
        img_path = os.path.join(self.image_dir, "{:06d}.png".format(sample_id))
        lidar = self.get_lidar(sample_id)
        calib = self.get_calib(sample_id)
        labels, has_labels = self.get_label(sample_id)
        if has_labels:
            labels[:, 1:] = transformation.camera_to_lidar_box(labels[:, 1:], calib.V2C, calib.R0, calib.P2)
        if self.lidar_aug:
            lidar, labels[:, 1:] = self.lidar_aug(lidar, labels[:, 1:])
        labels = filter_labels(labels, cnf.boundary)  # the points are filtered with the map
        hflipped = bool(np.random.random() < self.hflip_prob)
        targets = self.build_targets(labels, hflipped)
        return {"img_path": img_path, "hflipped": hflipped}, self._bev(lidar, hflipped), targets

    def get_image(self, idx):
        import cv2  # image decoding only (as the reference)
        img_path = os.path.join(self.image_dir, "{:06d}.png".format(idx))
        img = cv2.cvtColor(cv2.imread(img_path), cv2.COLOR_BGR2RGB)
        return img_path, img

    def get_calib(self, idx):
        from data_process.kitti_data_utils import Calibration
        return Calibration(os.path.join(self.calib_dir, "{:06d}.txt".format(idx)))

    def get_lidar(self, idx):
        lidar_file = os.path.join(self.lidar_dir, "{:06d}.bin".format(idx))
        return np.fromfile(lidar_file, dtype=np.float32).reshape(-1, 4)

    def __getattr__(self, name):
        # reference training helpers (get_label, build_targets, draw_img_with_label, ...)
        if name.startswith("__") or name in ("defer_bev",):
            raise AttributeError(name)
        attr = getattr(_reference_class(), name)
        return attr.__get__(self, type(self)) if hasattr(attr, "__get__") else attr


__getattr__ = _dropin.module_getattr(__name__)
