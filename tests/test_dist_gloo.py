"""World-size-2 (gloo, CPU) coverage of the frame-sharded multi-GPU path.

The per-rank step is a deterministic CPU stand-in for the GPU pipeline (the
collective logic — sharding, padding, all-gather, reordering — is what is under
test here; the kernels are covered by the -m gpu tests)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sfa_hip import dist as sdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def fake_step(ids, K=5):
    """(len(ids), K, 10) detections whose values encode the frame id."""
    out = torch.zeros((len(ids), K, 10))
    for r, f in enumerate(ids):
        out[r, :, 0] = float(f)
        out[r, :, 1] = torch.arange(K, dtype=torch.float32)
    return out


def _worker(rank, world, port, num_frames, batch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d, i = sdist.run_sharded(lambda ids: fake_step(ids), num_frames, batch, 5, "cpu")
        q.put((rank, d.numpy(), i.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("num_frames,batch", [(40, 4), (37, 4), (3, 4)])
def test_sharded_gather_world2(num_frames, batch):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, num_frames, batch, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, d, i in res:
        np.testing.assert_array_equal(i, np.arange(num_frames))
        np.testing.assert_array_equal(d[:, 0, 0], np.arange(num_frames, dtype=np.float32))
        np.testing.assert_array_equal(d[:, :, 1], np.tile(np.arange(5, dtype=np.float32), (num_frames, 1)))


def test_shard_batches_partition():
    for n, b, w in [(100, 16, 8), (17, 16, 2), (1, 16, 4), (64, 16, 4)]:
        got = np.concatenate([np.concatenate(sdist.shard_batches(n, b, w, r) or [np.zeros(0, np.int64)])
                              for r in range(w)])
        np.testing.assert_array_equal(np.sort(got), np.arange(n))
        assert max(len(sdist.shard_batches(n, b, w, r)) for r in range(w)) == sdist.steps_per_rank(n, b, w)


def _worker_big_ids(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dets = torch.full((3, 4, 10), float(rank))
        ids = torch.tensor([2 ** 40 + rank, -1, 2 ** 24 + 1 + rank], dtype=torch.int64)
        d, i = sdist.gather_detections(dets, ids)
        q.put((rank, d.numpy(), i.numpy()))
    finally:
        dist.destroy_process_group()


def test_gather_packs_ids_exactly():
    """The one-collective gather bit-casts the int64 frame ids into the detection rows: ids beyond
    float32's integer range and the -1 padding marker come back exactly."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_big_ids, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, d, i in res:
        np.testing.assert_array_equal(i, [2 ** 40, -1, 2 ** 24 + 1, 2 ** 40 + 1, -1, 2 ** 24 + 2])
        assert d.shape == (6, 4, 10)
        np.testing.assert_array_equal(d[:3], 0.0)
        np.testing.assert_array_equal(d[3:], 1.0)
