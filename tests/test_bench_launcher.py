"""bench.py --gpus N > 1 without a launcher: the parent starts the ranks
itself, touches no GPU, forwards rank 0's single JSON line and propagates a failing rank's exit
status.  Exercised with --dry-run (gloo all-gathers of rank-coded detections, no GPU)."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT",
                        "SFA_BENCH_FAIL_RANK", "SFA_BENCH_LAUNCHER")}
    env.update(kw)
    return env


def _json_lines(out: str):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_dry_run(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run", "--steps", "4",
                        "--warmup", "1", "--batch", "3", "--K", "5"],
                       env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    ln = lines[0]
    assert ln["n_gpus"] == n and ln["steps"] == 4 and ln["warmup"] == 1 and ln["dry_run"]
    assert ln["config"]["launcher"] == "bench.py"
    assert ln["config"]["global_batch"] == 3 * n
    assert ln["value"] > 0 and ln["scaling"] == "weak"


@pytest.mark.parametrize("fail_rank", [0, 1])
def test_self_launch_propagates_failure(fail_rank):
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "50",
                        "--warmup", "1"], env=_env(SFA_BENCH_FAIL_RANK=str(fail_rank)),
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert _json_lines(r.stdout) == []
    assert f"rank {fail_rank}: SFA_BENCH_FAIL_RANK" in r.stderr


def test_external_launcher_still_works():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "2",
                        "--dry-run", "--steps", "3", "--warmup", "1"],
                       env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2
    assert lines[0]["config"]["launcher"] == "external"


def test_launcher_parent_touches_no_gpu(monkeypatch):
    """The parent reaches launch_ranks before any torch.cuda call or HIP library load."""
    sys.path.insert(0, REPO)
    import torch

    import bench
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)

    def boom(*a, **k):
        raise AssertionError("the launcher parent touched the GPU")

    for name in ("is_available", "set_device", "current_device", "synchronize", "_lazy_init",
                 "current_stream", "device_count"):
        monkeypatch.setattr(torch.cuda, name, boom)
    monkeypatch.setattr(bench._lib, "lib", boom)
    seen = {}

    def fake_launch(n, argv, poll_s=0.05):
        seen["n"], seen["argv"] = n, list(argv)
        return 0

    monkeypatch.setattr(bench, "launch_ranks", fake_launch)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    with pytest.raises(SystemExit) as ei:
        bench.main()
    assert ei.value.code == 0
    assert seen == {"n": 8, "argv": ["--gpus", "8", "--steps", "3"]}
