"""KITTI velodyne .bin streaming over sfa_bin_stream_* (include/sfa_hip.h).

The reference reads one file per item (data_process/kitti_dataset.py:119-122 get_lidar:
np.fromfile(path, float32).reshape(-1, 4)) and voxelises it on the CPU.  BinStream reads
whole batches with a native reader pool into pinned staging memory and DMAs each batch into
one resident device buffer, overlapped with the GPU work on the previous batch:

    with BinStream(paths, batch=16, max_points_per_batch=16 * 150_000, device="cuda:0") as s:
        for points, offsets in s:          # points: (N, 4) f32 on the GPU, offsets: np.int64
            pipe.load_points(points, offsets)
            dets = pipe.run()

``device=None`` streams into host memory instead (no GPU needed; used by the CPU tests).
"""

from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, lib


class BinStream:
    def __init__(self, paths, batch: int, max_points_per_batch: int, n_threads: int = 8,
                 device=None, n_buffers: int = 1):
        self.paths = [str(p) for p in paths]
        self.batch = int(batch)
        self.cap = int(max_points_per_batch)
        self.device = None if device is None else torch.device(device)
        arr = (ctypes.c_char_p * max(1, len(self.paths)))(*[p.encode() for p in self.paths])
        h = ctypes.c_void_p()
        check(lib().sfa_bin_stream_create(arr, len(self.paths), self.batch, self.cap, int(n_threads),
                                          0 if self.device is None else 1, ctypes.byref(h)),
              "sfa_bin_stream_create")
        self._h = h
        # resident destination buffers, used in turn (2: the next batch can be copied while
        # the previous one is still being voxelised)
        self.bufs = [torch.empty((self.cap, 4), dtype=torch.float32,
                                 device=self.device if self.device is not None else "cpu")
                     for _ in range(max(1, int(n_buffers)))]
        self.count = 0
        self._offs = (ctypes.c_int64 * (self.batch + 1))()

    def next(self, stream=None):
        """-> (points (N, 4) view of the next resident buffer, offsets (n_frames + 1,)) or
        None at the end.  Device mode: the copy is enqueued on ``stream``."""
        n = ctypes.c_int()
        st = None
        if self.device is not None:
            st = stream if stream is not None else _lib.stream_ptr(self.device)
        buf = self.bufs[self.count % len(self.bufs)]
        check(lib().sfa_bin_stream_next(self._h, buf.data_ptr(), self.cap, self._offs,
                                        ctypes.byref(n), st), "sfa_bin_stream_next")
        if n.value == 0:
            return None
        self.count += 1
        offs = np.array(self._offs[: n.value + 1], dtype=np.int64)
        return buf[: offs[-1]], offs

    def __iter__(self):
        while True:
            item = self.next()
            if item is None:
                return
            yield item

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().sfa_bin_stream_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class StreamingDetector:
    """.bin files -> (pinned DMA) -> BEV -> KFPN forward -> decode, one batch at a time, with
    the host reads and the H2D copy of batch k+1 overlapping the GPU work of batch k.

    ``inflight`` pipelines (each with its own buffers and model handle, ``KfpnEngine.twin``)
    take the batches in turn on their own streams; the forward + decode of each is a HIP graph
    (``graph=True``), the voxeliser (ragged per-batch frame offsets) is launched eagerly.
    Two pipelines need an engine without side streams (``KfpnEngine(..., side_streams=False)``;
    the twins inherit it): with the copy stream beside them, two pipelines' streams AND their
    side streams exceed HIP's 4 hardware queues per process and measured 7 % slower
    (profiles/r02_stream_variants.txt); without side streams two pipelines are 13 % faster than
    one (profiles/r02b_stream_side_streams.txt: 4,440 -> 5,010 frames/s). Default 1.

    ``run(callback)`` calls ``callback(dets_view, n_frames, batch_index)`` after each batch
    is enqueued, with that batch's stream current (dets are valid once that stream reaches
    that point; work the callback enqueues there is ordered before the pipeline's reuse)."""

    def __init__(self, engine, paths, batch: int = 16, K: int = 50, n_threads: int = 8,
                 max_points_per_frame: int = 200_000, inflight: int = 1, graph: bool = True):
        from .runtime import DetectorPipeline
        self.dev = engine.device
        self.batch = batch
        engines = [engine] + [engine.twin() for _ in range(max(1, int(inflight)) - 1)]
        self.pipes = [DetectorPipeline(e, batch, K=K, with_bev=True, max_points=1) for e in engines]
        if graph:
            for p in self.pipes:
                p.capture_infer()
        self.src = BinStream(paths, batch, batch * max_points_per_frame, n_threads, self.dev,
                             n_buffers=2)

    @property
    def pipe(self):
        return self.pipes[0]

    def run(self, callback=None):
        with torch.cuda.device(self.dev):
            main = torch.cuda.current_stream()
            comps = [main] + [torch.cuda.Stream() for _ in range(len(self.pipes) - 1)]
            for c in comps[1:]:
                c.wait_stream(main)
            copy = torch.cuda.Stream()
            nb = len(self.src.bufs)
            ev_copy = [torch.cuda.Event() for _ in range(nb)]
            ev_bev = [torch.cuda.Event() for _ in range(nb)]
            item = self.src.next(copy.cuda_stream)
            ev_copy[0].record(copy)
            k = 0
            while item is not None:
                pts, offs = item
                pipe, comp = self.pipes[k % len(self.pipes)], comps[k % len(comps)]
                with torch.cuda.stream(comp):
                    comp.wait_event(ev_copy[k % nb])
                    pipe.load_points(pts, offs)
                    pipe.run(bev_done=ev_bev[k % nb])
                    if callback is not None:
                        callback(pipe.dets, len(offs) - 1, k)
                # buffer (k + 1) % nb is free once the BEV pass of batch k + 1 - nb is done
                if k + 1 >= nb:
                    copy.wait_event(ev_bev[(k + 1) % nb])
                item = self.src.next(copy.cuda_stream)
                ev_copy[(k + 1) % nb].record(copy)
                k += 1
            for c in comps[1:]:
                main.wait_stream(c)
            return k

    def close(self):
        self.src.close()
