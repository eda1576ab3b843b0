"""Drop-in for the reference's data_process/kitti_dataloader.py (:18-56).

``create_test_dataloader`` / ``create_val_dataloader`` / ``create_train_dataloader`` keep the
reference's signatures, DataLoader settings (batch size, shuffle, ``pin_memory``, ``num_workers``,
``DistributedSampler``) and batch structure, with one difference in WHERE the BEV maps are made:
the workers only read files (``kitti_dataset.KittiDataset`` with ``defer_bev``), and each batch's
sweeps are voxelised on the GPU in the main process — one ``sfa_bev_voxelize`` launch per batch
(the get_filtered_lidar box test fused in), in the reference's map layout and dtype: a
(B, 3, 608, 608) float64 CPU tensor, bit-exact with ``torch.from_numpy(makeBEVMap(...))`` stacked by
the default collate (``test.py:124`` then moves it to the device and casts it, ``:127`` reads it as
numpy for drawing).  Workers never touch HIP, so the callers' order — model on the GPU first
(``test.py:112``), then the loader (``:120``) with ``--num_workers 1`` — works.

Opt-in ``configs.bev_on_device = True`` (default False: the reference's f64 CPU tensor): the maps
are yielded as a (B, 3, 608, 608) float32 tensor already on the GPU — the voxeliser writes the
model's input layout directly, so the 8.9 MB-per-frame f64 device-to-host copy and the caller's
host-to-device copy back (``test.py:124`` ``.to(device).float()``, then a no-op) disappear.  The
values are the f64 maps rounded to float32, i.e. what ``.float()`` makes of the default tensor, so
detections are bit-equal in both modes.  For callers that do not read the maps as numpy.
"""

from __future__ import annotations

import numpy as np
import torch
from torch.utils.data import DataLoader
from torch.utils.data._utils.collate import default_collate

import config.kitti_config as cnf
from data_process.kitti_dataset import DeferredBEV, KittiDataset
from sfa_hip import _lib, runtime
from sfa_hip import dropin as _dropin


class DeferredBEVBatch:
    """The DeferredBEV samples of one batch (collated in the worker without touching them)."""

    __slots__ = ("items",)

    def __init__(self, items):
        self.items = list(items)

    def __reduce__(self):
        return DeferredBEVBatch, (self.items,)

    def voxelize(self, device=None, boundary=None, on_device: bool = False) -> torch.Tensor:
        """(B, 3, 608, 608) float64 CPU tensor: every sweep's map (get_filtered_lidar + makeBEVMap),
        made on the GPU ``device`` (default: the current one) in launches of up to 64 sweeps.
        ``on_device``: the same maps as a float32 tensor left on that GPU (module docstring)."""
        dev = runtime.host_api_device("the loader's BEV maps", device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        boundary = boundary or cnf.boundary
        shape = (len(self.items), 3, cnf.BEV_HEIGHT, cnf.BEV_WIDTH)
        if on_device:
            out = torch.empty(shape, dtype=torch.float32, device=dev)
            layout = _lib.BEV_NCHW3_F32
        else:
            out = torch.empty(shape, dtype=torch.float64)
            layout = _lib.BEV_NCHW3_F64
        vox = runtime.voxelizer(dev)
        for c0 in range(0, len(self.items), _lib.SFA_BEV_MAX_BATCH):
            chunk = self.items[c0:c0 + _lib.SFA_BEV_MAX_BATCH]
            offs = np.cumsum([0] + [d.points.shape[0] for d in chunk])
            pts = np.concatenate([d.points for d in chunk]) if offs[-1] else np.zeros((1, 4), np.float32)
            if on_device:  # written in place: no intermediate map
                vox(torch.from_numpy(pts).to(dev), offs, boundary, layout=layout, flags=_lib.BEV_RAW,
                    out=out[c0:c0 + len(chunk)])
            else:
                maps = vox(torch.from_numpy(pts).to(dev), offs, boundary, layout=layout, flags=_lib.BEV_RAW)
                out[c0:c0 + len(chunk)].copy_(maps)
        for i, d in enumerate(self.items):
            if d.flip_w:  # train-mode hflip: torch.flip(bev_map, [-1]) (kitti_dataset.py:97)
                out[i] = torch.flip(out[i], [-1])
        return out


def bev_collate(batch):
    """default_collate for every field except the DeferredBEV ones, which are kept as a
    DeferredBEVBatch for the main process (runs in the workers: no HIP)."""
    first = batch[0]
    if isinstance(first, (tuple, list)):
        cols = list(zip(*batch))
        return type(first)(DeferredBEVBatch(c) if isinstance(c[0], DeferredBEV) else default_collate(list(c))
                           for c in cols)
    if isinstance(first, DeferredBEV):
        return DeferredBEVBatch(batch)
    return default_collate(batch)


class DeviceBEVLoader:
    """Iterates the wrapped DataLoader and resolves each batch's DeferredBEVBatch into its BEV maps
    (DeferredBEVBatch.voxelize) in the calling (main) process.  Everything else — len(), .dataset,
    .batch_size, .sampler, ... — is the DataLoader's."""

    def __init__(self, loader: DataLoader, device=None, on_device: bool = False):
        self.loader = loader
        self.device = device
        self.on_device = bool(on_device)

    def __iter__(self):
        dev, od = self.device, self.on_device
        for batch in self.loader:
            if isinstance(batch, (tuple, list)):
                yield type(batch)(b.voxelize(dev, on_device=od) if isinstance(b, DeferredBEVBatch) else b
                                  for b in batch)
            elif isinstance(batch, DeferredBEVBatch):
                yield batch.voxelize(dev, on_device=od)
            else:
                yield batch

    def __len__(self):
        return len(self.loader)

    def __getattr__(self, name):
        if name in ("loader", "device", "on_device"):
            raise AttributeError(name)
        return getattr(self.loader, name)


def _cfg(configs, name, default):
    """configs.<name>, or default when unset (EasyDict raises AttributeError, dict-backed configs
    KeyError)."""
    try:
        return getattr(configs, name)
    except (AttributeError, KeyError):
        return default


def _loader(dataset, configs, shuffle, sampler):
    dataset.defer_bev = True
    on_device = bool(_cfg(configs, "bev_on_device", False))  # opt-in (module docstring)
    device = _cfg(configs, "device", None) if on_device else None
    if device is not None and torch.device(device).type != "cuda":
        # the device-resident maps live on a GPU: a CPU configs.device (--no_cuda) with bev_on_device is a
        # contradiction, not a request for the current GPU
        raise ValueError(f"configs.bev_on_device needs a CUDA configs.device, got {device}: unset bev_on_device "
                         "for the reference's float64 CPU maps")
    return DeviceBEVLoader(DataLoader(dataset, batch_size=configs.batch_size, shuffle=shuffle,
                                      pin_memory=configs.pin_memory, num_workers=configs.num_workers,
                                      sampler=sampler, collate_fn=bev_collate), device=device, on_device=on_device)


def create_train_dataloader(configs):
    """Create dataloader for training (kitti_dataloader.py:18-32)."""
    from data_process.transformation import OneOf, Random_Rotation, Random_Scaling
    train_lidar_aug = OneOf([
        Random_Rotation(limit_angle=np.pi / 4, p=1.0),
        Random_Scaling(scaling_range=(0.95, 1.05), p=1.0),
    ], p=0.66)
    train_dataset = KittiDataset(configs, mode="train", lidar_aug=train_lidar_aug, hflip_prob=configs.hflip_prob,
                                 num_samples=configs.num_samples)
    train_sampler = None
    if configs.distributed:
        train_sampler = torch.utils.data.distributed.DistributedSampler(train_dataset)
    return _loader(train_dataset, configs, train_sampler is None, train_sampler), train_sampler


def create_val_dataloader(configs):
    """Create dataloader for validation (kitti_dataloader.py:35-43)."""
    val_sampler = None
    val_dataset = KittiDataset(configs, mode="val", lidar_aug=None, hflip_prob=0., num_samples=configs.num_samples)
    if configs.distributed:
        val_sampler = torch.utils.data.distributed.DistributedSampler(val_dataset, shuffle=False)
    return _loader(val_dataset, configs, False, val_sampler)


def create_test_dataloader(configs):
    """Create dataloader for testing phase (kitti_dataloader.py:46-56)."""
    test_dataset = KittiDataset(configs, mode="test", lidar_aug=None, hflip_prob=0., num_samples=configs.num_samples)
    test_sampler = None
    if configs.distributed:
        test_sampler = torch.utils.data.distributed.DistributedSampler(test_dataset)
    return _loader(test_dataset, configs, False, test_sampler)


__getattr__ = _dropin.module_getattr(__name__)
