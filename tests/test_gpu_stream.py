"""Device side of the .bin streaming row: batches DMA'd from pinned staging
equal np.fromfile of the files, and the streaming detector (reads + H2D overlapped with the
GPU work of the previous batch) produces exactly the detections of the resident-buffer
pipeline on the same clouds."""
import numpy as np
import pytest
import torch

import golden_cases as gc
from sfa_hip import _lib, runtime, synthetic
from sfa_hip.stream import BinStream, StreamingDetector

pytestmark = pytest.mark.gpu


def test_device_stream_matches_fromfile(tmp_path, gpu):
    rng = np.random.default_rng(3)
    paths = []
    for i, n in enumerate([5000, 0, 70000, 12345, 1, 33333, 4096]):
        p = tmp_path / f"{i:06d}.bin"
        rng.standard_normal((n, 4)).astype(np.float32).tofile(p)
        paths.append(p)
    with BinStream(paths, 3, 200_000, n_threads=4, device=gpu, n_buffers=2) as s:
        i = 0
        for pts, offs in s:
            host = pts.cpu().numpy()
            for j in range(len(offs) - 1):
                ref = np.fromfile(paths[i], dtype=np.float32).reshape(-1, 4)
                np.testing.assert_array_equal(host[offs[j]:offs[j + 1]], ref)
                i += 1
        assert i == len(paths)


@pytest.mark.parametrize("inflight,graph,side", [(1, True, True), (1, False, True), (2, True, True),
                                                 (2, True, False)])
def test_streaming_detector_matches_pipeline(tmp_path, golden, gpu, inflight, graph, side):
    """Every configuration (forward + decode as a HIP graph or eager; 1 or 2 pipelines in flight,
    the second on a twin model handle over the same weights; with or without the models' side
    streams, as bench.py's stream workload runs 2 pipelines) == the eager resident pipeline."""
    clouds = [synthetic.synthetic_point_cloud(s) for s in range(1, 6)]  # 5 frames, batch 2
    paths = []
    for i, c in enumerate(clouds):
        p = tmp_path / f"{i:06d}.bin"
        c.tofile(p)
        paths.append(p)
    arch = _lib.make_arch(gc.HEADS)
    eng = runtime.KfpnEngine(arch, runtime.pack_state_dict(gc.state_dict_np(golden.model), arch), gpu,
                             side_streams=side)
    got = []
    sd = StreamingDetector(eng, paths, batch=2, K=50, n_threads=2, inflight=inflight, graph=graph)
    sd.run(lambda dets, n, k: got.append(dets[:n].clone()))
    torch.cuda.synchronize()
    sd.close()
    got = torch.cat(got).cpu().numpy()
    assert got.shape == (5, 50, 10)
    ref = []
    for k in range(0, 5, 2):
        chunk = clouds[k:k + 2]
        pipe = runtime.DetectorPipeline(eng, 2, K=50, with_bev=True,
                                        max_points=sum(c.shape[0] for c in chunk) + 200_000)
        pipe.set_points(chunk + [np.zeros((0, 4), np.float32)] * (2 - len(chunk)))
        ref.append(pipe.run()[: len(chunk)].cpu().numpy())
    np.testing.assert_array_equal(got, np.concatenate(ref))
