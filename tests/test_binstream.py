"""sfa_bin_stream in host mode: every batch equals
np.fromfile(path, float32).reshape(-1, 4) (data_process/kitti_dataset.py:119-122) of its
files, concatenated; ragged files, empty files, a partial last batch and the reference's
reshape error.  CPU only (the device copy is covered by tests/test_gpu_stream.py)."""
import numpy as np
import pytest

from sfa_hip import SfaNativeError
from sfa_hip.stream import BinStream


def _write(tmp_path, sizes, seed=0):
    rng = np.random.default_rng(seed)
    paths, clouds = [], []
    for i, n in enumerate(sizes):
        c = rng.standard_normal((n, 4)).astype(np.float32)
        p = tmp_path / f"{i:06d}.bin"
        c.tofile(p)
        paths.append(p)
        clouds.append(c)
    return paths, clouds


@pytest.mark.parametrize("batch,threads", [(4, 3), (16, 8), (1, 1)])
def test_stream_matches_fromfile(tmp_path, batch, threads):
    sizes = [1000, 0, 131072, 7, 50000, 1, 99999, 123457, 5, 60000, 3]
    paths, clouds = _write(tmp_path, sizes)
    got = []
    with BinStream(paths, batch, max_points_per_batch=sum(sizes), n_threads=threads) as s:
        for pts, offs in s:
            assert len(offs) - 1 <= batch
            for i in range(len(offs) - 1):
                got.append(pts[offs[i]:offs[i + 1]].numpy().copy())
    assert len(got) == len(sizes)
    for g, p in zip(got, paths):
        np.testing.assert_array_equal(g, np.fromfile(p, dtype=np.float32).reshape(-1, 4))


def test_trailing_bytes_and_reshape_error(tmp_path):
    paths, _ = _write(tmp_path, [10, 20])
    with open(paths[0], "ab") as f:
        f.write(b"\x00\x01")  # < one float: ignored by fromfile
    with BinStream(paths, 2, 100) as s:
        pts, offs = s.next()
        assert list(offs) == [0, 10, 30]
    with open(paths[1], "ab") as f:
        f.write(np.zeros(3, np.float32).tobytes())  # 83 floats: reshape(-1, 4) raises
    with pytest.raises(ValueError):
        np.fromfile(paths[1], dtype=np.float32).reshape(-1, 4)
    with BinStream(paths, 2, 100) as s, pytest.raises(SfaNativeError):
        s.next()


def test_capacity_and_missing_file(tmp_path):
    paths, _ = _write(tmp_path, [100, 100])
    with BinStream(paths, 2, 150) as s, pytest.raises(SfaNativeError, match="max_points"):
        s.next()
    with BinStream([tmp_path / "nope.bin"], 1, 10) as s, pytest.raises(SfaNativeError, match="stat"):
        s.next()
    with BinStream([], 4, 10) as s:
        assert s.next() is None


SANITIZERS = {"asan_ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"],
              "tsan": ["-fsanitize=thread"]}


@pytest.mark.parametrize("san", sorted(SANITIZERS))
def test_binstream_under_host_sanitizers(tmp_path, san):
    """csrc/binstream.cpp (producer thread + pread pool + two-slot state machine) built with
    ASan + UBSan and with TSan and driven by tests/native/binstream_sanitize.cpp in host mode:
    batches equal the files' bytes for several batch / reader counts, early destroy, error
    batches; any sanitizer report fails the run (SURVEY §5 race detection)."""
    import os
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None or not os.path.isdir("/opt/rocm/include"):
        pytest.skip("g++ / ROCm headers not available")
    here = os.path.dirname(os.path.abspath(__file__))
    csrc = os.path.join(os.path.dirname(here), "lidar-image_object-detection_-fpn_resnet-yolov8_amd", "csrc")
    exe = str(tmp_path / f"binstream_{san}")
    cmd = [gxx, "-std=c++17", "-g", "-O1", "-fno-omit-frame-pointer", *SANITIZERS[san],
           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", os.path.join(csrc, "binstream.cpp"),
           os.path.join(here, "native", "binstream_sanitize.cpp"), "-L/opt/rocm/lib",
           "-Wl,-rpath,/opt/rocm/lib", "-lamdhip64", "-pthread", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "binstream sanitize ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
