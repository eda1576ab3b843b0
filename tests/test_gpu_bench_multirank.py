"""configs[3] on the GPU: ``bench.py --gpus 2`` as a fresh subprocess, the
parent self-launching both ranks before any GPU call, both ranks sharing the one GPU of the test
box (``SFA_BENCH_SHARE_DEVICE=1``) and joined by gloo (``SFA_DIST_BACKEND=gloo``: RCCL refuses two
ranks on one device).  Everything else is the N > 1 path the driver's 8-GPU run takes: the timed
``BevInferBench`` at world 2 (2 pipelines per rank, HIP graphs, side streams off), rank r's frames
``synthetic_bev(16, seed=1 + r)`` with ids r*16 .. r*16+15, one packed all-gather per step
(``sfa_hip.dist.gather_detections``), the max-over-ranks JSON line.

``--dump-dets`` makes rank 0 write the gathered (2*16, 50, 10) detections and ids of one more step
per pipeline; they must equal, bit for bit, two single-rank pipelines built here with bench's own
``build_pipeline`` for ranks 0 and 1 (world 1, side streams on: the stream layout does not change
a bit), with every id exact.  Reference: the multi-process entry of train.py:58-67,82-83 and
models/model_utils.py:56-82 (DDP set-up), here for frame-parallel inference."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import bench

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT",
                        "SFA_BENCH_FAIL_RANK", "SFA_BENCH_LAUNCHER")}
    env.update(kw)
    return env


def test_bench_two_ranks_gather_equals_single_rank_pipelines(gpu, tmp_path):
    dump = str(tmp_path / "dets.npz")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "4",
                        "--warmup", "1", "--probe-forwards", "0", "--no-cpu-baseline", "--dump-dets", dump],
                       env=_env(SFA_BENCH_SHARE_DEVICE="1", SFA_DIST_BACKEND="gloo"),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["config"]["global_batch"] == 32 and ln["value"] > 0
    assert ln["config"]["side_streams"] is False and ln["config"]["steps_in_flight"] == 2
    got = np.load(dump)
    assert int(got["world"]) == 2 and int(got["side_streams"]) == 0
    dets, ids = got["dets"], got["ids"]
    assert dets.shape == (2, 32, 50, 10) and ids.shape == (2, 32)
    np.testing.assert_array_equal(ids, np.tile(np.arange(32, dtype=np.int64), (2, 1)))

    args = bench.parse([])
    for rank in range(2):
        assert int(got["input_seed"][rank]) == 1 + rank
        ref = bench.BevInferBench(args, rank, 1, gpu)
        assert ref.side is True
        for k in range(2):
            ref.one_step(k)
        torch.cuda.synchronize()
        exp = ref.pipes[0].dets.cpu().numpy()
        np.testing.assert_array_equal(ref.pipes[1].dets.cpu().numpy(), exp)
        for p in range(2):  # the step of each pipeline of the 2-rank run
            np.testing.assert_array_equal(dets[p, 16 * rank:16 * (rank + 1)], exp)
        del ref
        torch.cuda.empty_cache()


@pytest.mark.parametrize("workload", ["stream", "e2e"])
def test_bench_two_ranks_other_workloads_run(gpu, workload):
    """The other N > 1 paths of bench.py on the GPU (gloo, shared device): configs[3]'s .bin stream
    (each batch's detections all-gathered with frame ids, -1 padding) and configs[2]'s resident sweeps;
    both ranks finish and rank 0 prints one line with the whole-job frame count."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--workload", workload,
                        "--steps", "3", "--warmup", "1", "--probe-forwards", "0", "--no-cpu-baseline"],
                       env=_env(SFA_BENCH_SHARE_DEVICE="1", SFA_DIST_BACKEND="gloo"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2 and lines[0]["value"] > 0, r.stdout
    assert lines[0]["config"]["global_batch"] == 32
