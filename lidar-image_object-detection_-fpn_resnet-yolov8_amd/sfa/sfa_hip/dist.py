"""Frame-sharded multi-GPU inference: one process per GPU, no data-path collective.

Frames are independent (fpn_resnet.py:169-246, evaluation_utils.py:77-105), so a
KITTI stream is split into batches of ``batch`` consecutive frames and batch j is
owned by rank j % world.  Each rank voxelises, infers and decodes its own frames;
the only collective is one RCCL (backend "nccl" on ROCm) all-gather per step of the fixed
shape (B, K, 10) detections with their frame ids packed into the same rows.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_batches(num_frames: int, batch: int, world: int, rank: int):
    """Frame-index arrays (one per step) owned by `rank`; the last batch may be short."""
    out = []
    for j, start in enumerate(range(0, num_frames, batch)):
        if j % world == rank:
            out.append(np.arange(start, min(start + batch, num_frames), dtype=np.int64))
    return out


def steps_per_rank(num_frames: int, batch: int, world: int) -> int:
    nb = (num_frames + batch - 1) // batch
    return (nb + world - 1) // world


def gather_detections(dets: torch.Tensor, frame_ids: torch.Tensor, group=None):
    """All-gather (B, K, 10) float32 detections and (B,) int64 frame ids (-1 = padding) as ONE
    collective: each frame's row is its K*10 floats followed by its id's 8 bytes (bit-cast,
    so every id survives exactly), B * (K*10 + 2) * 4 bytes per rank.

    Returns (world*B, K, 10) and (world*B,) on every rank, rank-major."""
    world = dist.get_world_size(group)
    if world == 1:
        return dets, frame_ids
    if dets.dtype != torch.float32 or frame_ids.dtype != torch.int64:
        raise TypeError("gather_detections: float32 detections and int64 frame ids")
    B = dets.shape[0]
    row = dets[0].numel()
    packed = torch.cat([dets.reshape(B, row), frame_ids.contiguous().view(torch.float32).view(B, 2)], 1)
    out = torch.empty((world * B, row + 2), dtype=torch.float32, device=dets.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, packed, group=group)
    else:  # gloo (CPU tests / single-GPU rehearsal): gather through host memory
        oc = out.cpu()
        dist.all_gather(list(oc.chunk(world)), packed.cpu(), group=group)
        out.copy_(oc)
    d = out[:, :row].reshape((world * B,) + tuple(dets.shape[1:]))
    ids = out[:, row:].contiguous().view(torch.int64).reshape(world * B)
    return d, ids


def order_by_frame(dets: torch.Tensor, ids: torch.Tensor):
    """Drop padding rows and sort gathered detections by frame id."""
    keep = ids >= 0
    d, i = dets[keep], ids[keep]
    order = torch.argsort(i)
    return d[order], i[order]


def run_sharded(step_fn, num_frames: int, batch: int, K: int, device, group=None):
    """Drive `step_fn(frame_ids: np.ndarray) -> (len(ids), K, 10) tensor` over this rank's
    shards and gather everything; every rank returns all frames' detections in order."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    mine = shard_batches(num_frames, batch, world, rank)
    n_steps = steps_per_rank(num_frames, batch, world)
    all_d, all_i = [], []
    for s in range(n_steps):
        ids = mine[s] if s < len(mine) else np.zeros(0, np.int64)
        dets = torch.zeros((batch, K, 10), dtype=torch.float32, device=device)
        fid = torch.full((batch,), -1, dtype=torch.int64, device=device)
        if ids.size:
            dets[: ids.size] = step_fn(ids)
            fid[: ids.size] = torch.from_numpy(ids).to(device)
        if world > 1:
            g, gi = gather_detections(dets, fid, group)
        else:
            g, gi = dets, fid
        all_d.append(g)
        all_i.append(gi)
    return order_by_frame(torch.cat(all_d), torch.cat(all_i))
