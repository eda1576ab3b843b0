"""Host runtime over the C ABI: weight packing, engines, device buffers, streams.

torch is used only as plumbing (device memory, the current HIP stream, graph
capture); every computation on the hot path is a libsfa_hip kernel.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import SfaNativeError, check, lib

DEFAULT_HEADS = {"hm_cen": 3, "cen_offset": 2, "direction": 2, "z_coor": 1, "dim": 3}
DEFAULT_BOUNDARY = {"minX": 0, "maxX": 50, "minY": -25, "maxY": 25, "minZ": -2.73, "maxZ": 1.27}
# config/kitti_config.py:35-42 boundary_back (demo_2_sides.py's rear view)
DEFAULT_BOUNDARY_BACK = {"minX": -50, "maxX": 0, "minY": -25, "maxY": 25, "minZ": -2.73, "maxZ": 1.27}


def _require_gpu_tensor(t: torch.Tensor, what: str, dtype=torch.float32) -> torch.Tensor:
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise SfaNativeError(f"{what}: the HIP path needs a tensor on a GPU device "
                             f"(got {getattr(t, 'device', type(t))}); there is no CPU fallback")
    if t.dtype != dtype:
        raise TypeError(f"{what}: expected {dtype}, got {t.dtype}")
    return t.contiguous()


def host_api_device(what: str, device=None) -> torch.device:
    """The GPU a numpy-in / numpy-out host API (makeBEVMap, get_filtered_lidar) runs on: ``device``
    or the current one. Raises SfaNativeError with the fix when no GPU is visible or when called in a
    process forked after HIP was initialised — a DataLoader worker of a caller that created its model
    first (test.py:112 then :120): HIP cannot be used there, and the drop-in's
    data_process.kitti_dataloader voxelises each batch in the main process instead."""
    if device is not None:
        return torch.device(device)
    if torch.cuda._is_in_bad_fork():
        raise SfaNativeError(
            f"{what} runs on the GPU (HIP), but this process was forked after HIP was initialised "
            "(a DataLoader worker): create the loader with the drop-in data_process.kitti_dataloader "
            "(create_test_dataloader / create_val_dataloader / create_train_dataloader: the workers only "
            "read files, the BEV maps are made per batch in the main process) or use num_workers=0")
    if not torch.cuda.is_available():
        raise SfaNativeError(f"{what} runs on the GPU (HIP); no GPU is visible")
    return torch.device("cuda", torch.cuda.current_device())


def _boundary_arr(boundary: dict):
    vals = [boundary[k] for k in ("minX", "maxX", "minY", "maxY", "minZ", "maxZ")]
    return (ctypes.c_double * 6)(*[float(v) for v in vals])


# ------------------------------------------------------------------ weights
def pack_state_dict(state: dict, arch) -> np.ndarray:
    """Reference-format state_dict (tensors or arrays) -> packed float32 host array."""
    L = lib()
    layout = _lib.state_layout(arch)
    parts = []
    for name, shape in layout:
        if name.endswith("num_batches_tracked"):
            continue
        if name not in state:
            raise KeyError(f"state_dict is missing {name}")
        v = state[name]
        v = v.detach().to("cpu", torch.float32).numpy() if isinstance(v, torch.Tensor) else np.asarray(
            v, np.float32)
        if tuple(v.shape) != tuple(shape):
            raise ValueError(f"{name}: shape {tuple(v.shape)} != {tuple(shape)}")
        parts.append(np.ascontiguousarray(v, np.float32).reshape(-1))
    flat = np.concatenate(parts) if parts else np.zeros(0, np.float32)
    nfl = L.sfa_state_floats(ctypes.byref(arch))
    if flat.size != nfl:
        raise ValueError(f"state has {flat.size} floats, expected {nfl}")
    packed = np.zeros(L.sfa_packed_floats(ctypes.byref(arch)), np.float32)
    check(L.sfa_pack_weights(ctypes.byref(arch), flat.ctypes.data, flat.size, packed.ctypes.data),
          "sfa_pack_weights")
    return packed


class KfpnEngine:
    """A device copy of the packed weights + an sfa_model handle + workspace cache."""

    def __init__(self, arch, packed_host: np.ndarray, device, math=None, side_streams: bool = True):
        self.arch = arch
        self.device = torch.device(device)
        self.heads = [(arch.head_names[j].value.decode(), int(arch.head_channels[j]))
                      for j in range(arch.num_heads)]
        self.weights = torch.from_numpy(packed_host).to(self.device)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):  # the model's side stream lives on this device
            check(lib().sfa_model_create(ctypes.byref(arch), self.weights.data_ptr(), ctypes.byref(h)),
                  "sfa_model_create")
        self._h = h
        self._ws = {}
        self.side_streams = True
        self.set_math(_lib.math_from_env() if math is None else math)
        if not side_streams:
            self.set_side_streams(False)

    def set_math(self, math: int):
        """_lib.MATH_FP16X3 (default), _lib.MATH_BF16X6 or _lib.MATH_F32 for every convolution."""
        check(lib().sfa_model_set_math(self._h, int(math)), "sfa_model_set_math")
        self.math = int(math)

    def set_option(self, key: int, value: int):
        """Kernel-choice option of this handle (_lib.OPT_*, include/sfa_hip.h sfa_model_option):
        A/B runs and the kernel-equivalence tests; the defaults are the production kernels."""
        with torch.cuda.device(self.device):
            check(lib().sfa_model_set_option(self._h, int(key), int(value)), "sfa_model_set_option")

    def get_option(self, key: int) -> int:
        v = ctypes.c_int()
        check(lib().sfa_model_get_option(self._h, int(key), ctypes.byref(v)), "sfa_model_get_option")
        return int(v.value)

    def set_side_streams(self, on: bool):
        """Side stream for the level-0 heads on (default) or off (sfa_model_set_side_streams):
        off when several forwards are kept in flight beside a copy stream, so the process's
        streams fit HIP's 4 hardware queues. Not while a forward of this engine is running."""
        with torch.cuda.device(self.device):
            check(lib().sfa_model_set_side_streams(self._h, 1 if on else 0), "sfa_model_set_side_streams")
        self.side_streams = bool(on)

    def twin(self) -> "KfpnEngine":
        """A second model handle over the SAME device weights (sfa_model_create does not copy
        them): its own side stream and events (or none, like this engine), so two forwards can be
        in flight (or captured in two graphs) on two streams. Workspaces are per engine /
        pipeline as usual."""
        t = object.__new__(KfpnEngine)
        t.arch, t.device, t.heads, t.weights = self.arch, self.device, self.heads, self.weights
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().sfa_model_create(ctypes.byref(self.arch), self.weights.data_ptr(), ctypes.byref(h)),
                  "sfa_model_create")
        t._h = h
        t._ws = {}
        t.side_streams = True
        t.set_math(self.math)
        if not self.side_streams:
            t.set_side_streams(False)
        for key in range(_lib.OPT_COUNT):  # the same kernel choices (every option key)
            if t.get_option(key) != self.get_option(key):
                t.set_option(key, self.get_option(key))
        return t

    def set_probe(self, flags: int):
        """Kernel probe (measurement only): _lib.PROBE_HEADS records timing events around each
        head-level launch of un-captured forwards; _lib.PROBE_SERIAL keeps every launch on the
        caller's stream. 0 turns it off."""
        check(lib().sfa_model_set_probe(self._h, int(flags)), "sfa_model_set_probe")

    def probe_times(self, levels: int = 3):
        """Durations (ms) of the head-level launches of the last probed forward (waits for them)."""
        ms = (ctypes.c_float * levels)()
        check(lib().sfa_model_probe_times(self._h, ms, levels), "sfa_model_probe_times")
        return [float(v) for v in ms]

    def __del__(self):
        try:
            if getattr(self, "_h", None) is not None and self._h.value:
                lib().sfa_model_destroy(self._h)
        except Exception:
            pass

    def workspace_bytes(self, B, H, W) -> int:
        return int(lib().sfa_forward_workspace_size(self._h, B, H, W))

    WORKSPACE_CACHE = 2  # streams whose forward workspace stays resident (LRU)

    def workspace(self, B, H, W, stream: int = None) -> torch.Tensor:
        """The forward workspace (activations + fp16x3 max slots) of forwards issued on
        ``stream`` without an explicit workspace.  Eager forwards on different streams get
        different buffers; the last ``WORKSPACE_CACHE`` streams keep theirs resident, and
        evicting or re-shaping an entry first waits for the device, so a forward still running
        on the old buffer never sees it reused.  Graph captures all issue on torch's capture
        stream, so graphs captured without an explicit workspace SHARE one buffer: two such
        graphs must not be replayed concurrently (DetectorPipeline owns its workspace instead)."""
        sk = int(stream) if stream is not None else _lib.stream_ptr(self.device)
        cur = self._ws.pop(sk, None)
        if cur is not None and cur[0] == (B, H, W):
            self._ws[sk] = cur  # most recently used last
            return cur[1]
        if cur is not None or len(self._ws) >= self.WORKSPACE_CACHE:
            torch.cuda.synchronize(self.device)
            del cur
            while len(self._ws) >= self.WORKSPACE_CACHE:
                self._ws.pop(next(iter(self._ws)))
        ws = torch.empty(self.workspace_bytes(B, H, W), dtype=torch.uint8, device=self.device)
        self._ws[sk] = ((B, H, W), ws)
        return ws

    def alloc_outputs(self, B, H, W):
        return {name: torch.empty((B, ch, H // 4, W // 4), dtype=torch.float32, device=self.device)
                for name, ch in self.heads}

    def forward_into(self, x: torch.Tensor, outs: dict, in_layout: int = _lib.IN_NCHW3,
                     workspace: torch.Tensor = None, stream: int = None) -> dict:
        if in_layout != _lib.IN_NHWC4:
            B, C, H, W = x.shape
            if C != 3:
                raise ValueError(f"expected (B, 3, H, W) input, got {tuple(x.shape)}")
        else:
            B, H, W, C = x.shape
            if C != 4:
                raise ValueError(f"expected (B, H, W, 4) input, got {tuple(x.shape)}")
        sp = stream if stream is not None else _lib.stream_ptr(self.device)
        ws = workspace if workspace is not None else self.workspace(B, H, W, sp)
        ptrs = (ctypes.c_void_p * len(self.heads))(*[outs[n].data_ptr() for n, _ in self.heads])
        check(lib().sfa_model_forward(self._h, x.data_ptr(), in_layout, B, H, W, ptrs, ws.data_ptr(),
                                      ws.numel(), sp), "sfa_model_forward")
        return outs

    def debug_views(self, ws: torch.Tensor, B, H, W) -> dict:
        """NCHW views of intermediate maps left in the workspace by the last forward."""
        L = lib()

        def nhwc(which, h, w, c):
            off = int(L.sfa_forward_buffer_offset(self._h, B, H, W, which))
            t = ws[off: off + B * h * w * c * 4].view(torch.float32).view(B, h, w, c)
            return t.permute(0, 3, 1, 2)

        v = {f"layer{i + 1}": nhwc(i, H >> (i + 2), W >> (i + 2), 64 << i) for i in range(4)}
        v["up_level2"] = nhwc(4, H // 8, W // 8, 256)
        v["up_level3"] = nhwc(5, H // 4, W // 4, 128)
        v["up_level4"] = nhwc(6, H // 4, W // 4, 64)
        nch = sum(c for _, c in self.heads)
        lv = []
        for k, (h, w) in enumerate(((H // 8, W // 8), (H // 4, W // 4), (H // 4, W // 4))):
            off = int(L.sfa_forward_buffer_offset(self._h, B, H, W, 7 + k))
            lv.append(ws[off: off + nch * B * h * w * 4].view(torch.float32).view(nch, B, h, w))
        levels, c0 = {}, 0
        for name, ch in self.heads:
            levels[name] = [t[c0:c0 + ch].permute(1, 0, 2, 3) for t in lv]
            c0 += ch
        v["levels"] = levels
        return v

    def forward(self, x: torch.Tensor, in_layout: int = _lib.IN_NCHW3) -> dict:
        x = _require_gpu_tensor(x, "PoseResNet.forward")
        if in_layout != _lib.IN_NHWC4:
            B, _, H, W = x.shape
        else:
            B, H, W, _ = x.shape
        if H % 32 or W % 32:
            raise ValueError(f"input H, W must be multiples of 32, got {H}x{W}")
        with torch.cuda.device(self.device):
            outs = self.alloc_outputs(B, H, W)
            return self.forward_into(x, outs, in_layout)


# --------------------------------------------------------------------- BEV
class BevVoxelizer:
    """sfa_bev_voxelize with its (self-cleaning) scratch kept resident."""

    def __init__(self, device, max_batch: int = 16, force_atomic: bool = None, strip8: bool = None):
        """force_atomic: the global-atomic kernels instead of the binned ones (same bits; A/B),
        default from env SFA_BEV_ATOMIC read once here (flag SFA_BEV_FORCE_ATOMIC per call);
        strip8: the one-pass path with 8-row strips (round 3a; A/B), env SFA_BEV_STRIP8."""
        self.device = torch.device(device)
        if force_atomic is None:
            force_atomic = os.environ.get("SFA_BEV_ATOMIC", "0") not in ("", "0")
        if strip8 is None:
            strip8 = os.environ.get("SFA_BEV_STRIP8", "0") not in ("", "0")
        self.force_atomic = bool(force_atomic)
        self.strip8 = bool(strip8)
        self.max_batch = 0
        self.scratch = None
        self._grow(max_batch)

    def _grow(self, b):
        if b <= self.max_batch:
            return
        if b > _lib.SFA_BEV_MAX_BATCH:
            raise ValueError(f"BEV batch {b} > {_lib.SFA_BEV_MAX_BATCH}")
        self.scratch = torch.zeros(int(lib().sfa_bev_scratch_size(b)), dtype=torch.uint8,
                                   device=self.device)
        self.max_batch = b

    def __call__(self, points: torch.Tensor, offsets, boundary=DEFAULT_BOUNDARY,
                 layout: int = _lib.BEV_NHWC4_F32, flags: int = _lib.BEV_RAW, out=None,
                 stream: int = None) -> torch.Tensor:
        points = _require_gpu_tensor(points, "makeBEVMap")
        if points.ndim != 2 or points.shape[1] != 4:
            raise ValueError(f"points must be (N, 4), got {tuple(points.shape)}")
        offs = np.asarray(offsets, dtype=np.int64)
        B = offs.size - 1
        if B < 1 or offs[-1] > points.shape[0] or offs[0] < 0 or np.any(np.diff(offs) < 0):
            raise ValueError("bad frame offsets")
        self._grow(B)
        if out is None:
            if layout == _lib.BEV_NHWC4_F32:
                out = torch.empty((B, 608, 608, 4), dtype=torch.float32, device=self.device)
            else:
                dt = torch.float64 if layout == _lib.BEV_NCHW3_F64 else torch.float32
                out = torch.empty((B, 3, 608, 608), dtype=dt, device=self.device)
        offs_c = (ctypes.c_int64 * (B + 1))(*offs.tolist())
        if self.force_atomic:
            flags |= _lib.BEV_FORCE_ATOMIC
        if self.strip8:
            flags |= _lib.BEV_STRIP8
        check(lib().sfa_bev_voxelize(points.data_ptr() if points.numel() else None, offs_c, B,
                                     _boundary_arr(boundary), flags, layout, out.data_ptr(),
                                     self.scratch.data_ptr(), self.scratch.numel(),
                                     stream if stream is not None else _lib.stream_ptr(self.device)),
              "sfa_bev_voxelize")
        return out


_voxelizers = {}


def voxelizer(device) -> BevVoxelizer:
    device = torch.device(device)
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    v = _voxelizers.get(device)
    if v is None:
        v = _voxelizers[device] = BevVoxelizer(device)
    return v


def filter_points(points: torch.Tensor, boundary=DEFAULT_BOUNDARY) -> torch.Tensor:
    """get_filtered_lidar on the device: (N, 4) f32 -> (M, 4) f32 (order kept, z -= minZ)."""
    points = _require_gpu_tensor(points, "get_filtered_lidar")
    n = points.shape[0]
    out = torch.empty((max(n, 1), 4), dtype=torch.float32, device=points.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=points.device)
    scratch = torch.empty(int(lib().sfa_filter_scratch_size(n)), dtype=torch.uint8,
                          device=points.device)
    check(lib().sfa_filter_points(points.data_ptr() if n else None, n, _boundary_arr(boundary),
                                  out.data_ptr(), cnt.data_ptr(), scratch.data_ptr(), scratch.numel(),
                                  _lib.stream_ptr(points.device)), "sfa_filter_points")
    m = int(cnt.item())
    return out[:m]


# ------------------------------------------------------------------ decode
def sigmoid_clamp_(x: torch.Tensor) -> torch.Tensor:
    """_sigmoid (utils/torch_utils.py:44-45) in place on a float32 GPU tensor; a non-contiguous
    one (the reference accepts any strided tensor) goes through a contiguous copy that is
    written back into it."""
    if not isinstance(x, torch.Tensor) or x.device.type != "cuda" or x.dtype != torch.float32:
        raise SfaNativeError("_sigmoid: the HIP path needs a float32 GPU tensor")
    if x.numel() == 0:
        return x
    t = x if x.is_contiguous() else x.contiguous()
    check(lib().sfa_sigmoid_clamp_inplace(t.data_ptr(), t.numel(), _lib.stream_ptr(x.device)),
          "sfa_sigmoid_clamp_inplace")
    if t is not x:
        x.copy_(t)
    return x


def heat_nms(heat: torch.Tensor) -> torch.Tensor:
    """_nms (evaluation_utils.py:21-26, kernel 3): a new tensor heat * (max_pool3x3(heat) == heat)."""
    heat = _require_gpu_tensor(heat, "_nms")
    if heat.dim() < 2:
        raise ValueError("_nms: expected (..., H, W)")
    H, W = int(heat.shape[-2]), int(heat.shape[-1])
    out = torch.empty_like(heat)
    check(lib().sfa_heat_nms(heat.data_ptr() if heat.numel() else None, out.data_ptr() if out.numel() else None,
                             heat.numel() // max(1, H * W), H, W, _lib.stream_ptr(heat.device)), "sfa_heat_nms")
    return out


def topk(scores: torch.Tensor, K: int = 40, per_channel: bool = False):
    """_topk (evaluation_utils.py:47-62): (score (B,K) f32, inds (B,K) int64, clses (B,K) int32,
    ys (B,K) f32, xs (B,K) f32); per_channel = _topk_channel (:65-74): (scores, inds, ys, xs), each
    (B, C, K). Ties: lower flat index first, then lower class (torch leaves them unspecified)."""
    scores = _require_gpu_tensor(scores, "_topk")
    if scores.dim() != 4:
        raise ValueError(f"_topk: expected (B, C, H, W), got {tuple(scores.shape)}")
    B, C, H, W = (int(v) for v in scores.shape)
    K = int(K)
    if K > H * W:  # torch.topk: "selected index k out of range"
        raise RuntimeError(f"_topk: K = {K} exceeds the {H * W} elements of a class map")
    dev = scores.device
    shp = (B, C, K) if per_channel else (B, K)
    sc = torch.empty(shp, dtype=torch.float32, device=dev)
    ind = torch.empty(shp, dtype=torch.int64, device=dev)
    cls = None if per_channel else torch.empty(shp, dtype=torch.int32, device=dev)
    ys = torch.empty(shp, dtype=torch.float32, device=dev)
    xs = torch.empty(shp, dtype=torch.float32, device=dev)
    ws = torch.empty(int(lib().sfa_topk_workspace_size(B, C, K)), dtype=torch.uint8, device=dev)
    check(lib().sfa_topk(scores.data_ptr(), B, C, H, W, K, 1 if per_channel else 0, sc.data_ptr(), ind.data_ptr(),
                         cls.data_ptr() if cls is not None else None, ys.data_ptr(), xs.data_ptr(), ws.data_ptr(),
                         ws.numel(), _lib.stream_ptr(dev)), "sfa_topk")
    return (sc, ind, ys, xs) if per_channel else (sc, ind, cls, ys, xs)


def gather_feat(feat: torch.Tensor, ind: torch.Tensor, transpose: bool = False) -> torch.Tensor:
    """_gather_feat (evaluation_utils.py:29-37, mask None): feat (B, N, D), ind (B, K) int64 ->
    (B, K, D); transpose = _transpose_and_gather_feat (:40-44): feat (B, D, H, W) -> (B, K, D).
    4- or 8-byte elements (f32, int32, int64). Indices outside [0, N) raise, as torch.gather does."""
    if not isinstance(feat, torch.Tensor) or feat.device.type != "cuda":
        raise SfaNativeError("_gather_feat: the HIP path needs GPU tensors; there is no CPU fallback")
    if feat.element_size() not in (4, 8):
        raise TypeError(f"_gather_feat: {feat.dtype} elements are not 4 or 8 bytes")
    ind = _require_gpu_tensor(ind, "_gather_feat indices", torch.int64)
    feat = feat.contiguous()
    if transpose:
        if feat.dim() != 4:
            raise ValueError("_transpose_and_gather_feat: expected feat (B, C, H, W)")
        B, D, H, W = (int(v) for v in feat.shape)
        N, sn, sd = H * W, 1, H * W
    else:
        if feat.dim() != 3:
            raise ValueError("_gather_feat: expected feat (B, N, D)")
        B, N, D = (int(v) for v in feat.shape)
        sn, sd = D, 1
    if ind.dim() != 2 or int(ind.shape[0]) != B:
        raise ValueError(f"_gather_feat: indices {tuple(ind.shape)} do not match batch {B}")
    K = int(ind.shape[1])
    out = torch.empty((B, K, D), dtype=feat.dtype, device=feat.device)
    if ind.numel():
        lo, hi = (int(v) for v in torch.aminmax(ind))
        if lo < 0 or hi >= N:
            raise RuntimeError(f"_gather_feat: index {lo if lo < 0 else hi} is out of bounds for size {N}")
    check(lib().sfa_gather_feat(feat.data_ptr() if feat.numel() else None, B, N, D, sn, sd, feat.element_size(),
                                ind.data_ptr() if ind.numel() else None, K, out.data_ptr() if out.numel() else None,
                                _lib.stream_ptr(feat.device)), "sfa_gather_feat")
    return out


class Decoder:
    """sfa_decode with a workspace cached per (device, stream, shape): decodes on different
    streams never share scratch."""

    def __init__(self):
        self._ws = {}

    @staticmethod
    def workspace_bytes(B, C, K) -> int:
        return int(lib().sfa_decode_workspace_size(B, C, K))

    def workspace(self, device, B, C, K, stream: int = None):
        sk = int(stream) if stream is not None else _lib.stream_ptr(device)
        key = (str(device), sk, B, C, K)
        ws = self._ws.get(key)
        if ws is None:
            ws = torch.empty(self.workspace_bytes(B, C, K), dtype=torch.uint8, device=device)
            self._ws[key] = ws
        return ws

    def __call__(self, hm, off, dirn, z, dim, K=40, apply_sigmoid=False, out=None,
                 stream: int = None, workspace: torch.Tensor = None):
        hm = _require_gpu_tensor(hm, "decode")
        dirn, z, dim = (_require_gpu_tensor(t, "decode") for t in (dirn, z, dim))
        if off is not None:
            off = _require_gpu_tensor(off, "decode")
        B, C, H, W = hm.shape
        for t, c in ((off, 2), (dirn, 2), (z, 1), (dim, 3)):
            if t is not None and tuple(t.shape) != (B, c, H, W):
                raise ValueError(f"decode: map shape {tuple(t.shape)} != {(B, c, H, W)}")
        if out is None:
            out = torch.empty((B, K, 10), dtype=torch.float32, device=hm.device)
        sp = stream if stream is not None else _lib.stream_ptr(hm.device)
        ws = workspace if workspace is not None else self.workspace(hm.device, B, C, K, sp)
        if ws.numel() < self.workspace_bytes(B, C, K):
            raise ValueError("decode: workspace too small")
        check(lib().sfa_decode(hm.data_ptr(), off.data_ptr() if off is not None else None,
                               dirn.data_ptr(), z.data_ptr(), dim.data_ptr(), B, C, H, W, int(K),
                               1 if apply_sigmoid else 0, out.data_ptr(), ws.data_ptr(), ws.numel(),
                               sp),
              "sfa_decode")
        return out


_decoder = Decoder()


def decode(hm, off, dirn, z, dim, K=40, apply_sigmoid=False):
    return _decoder(hm, off, dirn, z, dim, K=K, apply_sigmoid=apply_sigmoid)


# ---------------------------------------------------------------- pipeline
class DetectorPipeline:
    """Fixed-shape hot path on one GPU: [points ->] BEV -> KFPN forward -> decode.

    All buffers are allocated once; ``run()`` only enqueues kernels on the current
    stream, so it can be captured in a HIP graph (``capture()``).
    """

    def __init__(self, engine: KfpnEngine, batch: int, height: int = 608, width: int = 608,
                 K: int = 50, with_bev: bool = False, max_points: int = 0, two_sided: bool = False,
                 boundary=DEFAULT_BOUNDARY, boundary_back=None, bev_layout: str = "nchw3"):
        """two_sided (with_bev only): every sweep is also voxelised with ``boundary_back``
        and flipped (demo_2_sides.py: demo_dataset.py:70-88 + demo_utils.py:110-111), so one
        run infers 2*batch maps: frames [0, batch) front, [batch, 2*batch) back.
        bev_layout (with_bev only): the voxeliser's output / the model's input — "nchw3" (the
        reference's (B, 3, 608, 608) f32, read by the patch stem directly: 3/4 of NHWC4's bytes)
        or "nhwc4" ((B, 608, 608, 4), channel 3 = 0)."""
        self.engine = engine
        self.dev = engine.device
        self.B, self.H, self.W, self.K = batch, height, width, K
        self.with_bev = with_bev
        self.two_sided = bool(two_sided)
        if self.two_sided and not with_bev:
            raise ValueError("two_sided needs with_bev (the back view is voxelised on the GPU)")
        self.boundary = boundary
        self.boundary_back = boundary_back if boundary_back is not None else DEFAULT_BOUNDARY_BACK
        nmap = 2 * batch if self.two_sided else batch
        self.nmap = nmap
        with torch.cuda.device(self.dev):
            # the pipeline's own workspace (it is replayed on streams of the caller's choosing,
            # so it must not be the engine's per-stream cache entry)
            self.ws = torch.empty(engine.workspace_bytes(nmap, height, width), dtype=torch.uint8,
                                  device=self.dev)
            self.outs = engine.alloc_outputs(nmap, height, width)
            self.dets = torch.empty((nmap, K, 10), dtype=torch.float32, device=self.dev)
            self.dec_ws = torch.empty(Decoder.workspace_bytes(nmap, dict(engine.heads)["hm_cen"], K),
                                      dtype=torch.uint8, device=self.dev)
            if with_bev:
                if (height, width) != (608, 608):
                    raise ValueError("the BEV grid is 608x608 (config/kitti_config.py:45-46)")
                self.vox = BevVoxelizer(self.dev, batch)
                if bev_layout not in ("nchw3", "nhwc4"):
                    raise ValueError(f"bev_layout must be 'nchw3' or 'nhwc4', not {bev_layout!r}")
                self.bev_layout = bev_layout
                self.bev_fmt = _lib.BEV_NCHW3_F32 if bev_layout == "nchw3" else _lib.BEV_NHWC4_F32
                self.in_fmt = _lib.IN_NCHW3 if bev_layout == "nchw3" else _lib.IN_NHWC4
                shape = (nmap, 3, 608, 608) if bev_layout == "nchw3" else (nmap, 608, 608, 4)
                self.bev = torch.empty(shape, dtype=torch.float32, device=self.dev)
                self.points = torch.zeros((max(max_points, 1), 4), dtype=torch.float32,
                                          device=self.dev)
                self.offsets = np.zeros(batch + 1, np.int64)
            else:
                self.x = torch.empty((batch, 3, height, width), dtype=torch.float32, device=self.dev)
        self.graph = None
        self.infer_graph = None  # forward + decode only (capture_infer): the BEV stays eager

    def set_points(self, clouds):
        """Copy a list of (N_i, 4) float32 clouds into the resident point buffer."""
        offs = np.zeros(len(clouds) + 1, np.int64)
        for i, c in enumerate(clouds):
            offs[i + 1] = offs[i] + c.shape[0]
        if len(clouds) != self.B or offs[-1] > self.points.shape[0]:
            raise ValueError("clouds do not fit the pipeline's point buffer")
        host = torch.from_numpy(np.concatenate(clouds).astype(np.float32))
        self.points[: offs[-1]].copy_(host)
        self.offsets = offs

    def load_points(self, points: torch.Tensor, offsets):
        """Use a resident device buffer of points (e.g. a BinStream batch) without a copy;
        a short batch is padded with empty frames."""
        offs = np.asarray(offsets, dtype=np.int64)
        if offs.size - 1 > self.B:
            raise ValueError("more frames than the pipeline batch")
        self.points = _require_gpu_tensor(points, "load_points")
        self.offsets = np.concatenate([offs, np.full(self.B + 1 - offs.size, offs[-1], np.int64)])

    def run(self, bev_done=None, _eager=False):
        """Enqueue the step; ``bev_done`` (torch.cuda.Event) is recorded once the points have
        been consumed (after voxelisation).  With ``capture_infer()`` done, the forward + decode
        part replays that graph (``_eager`` forces the eager launches: capture() uses it)."""
        st = _lib.stream_ptr(self.dev)
        if self.with_bev:
            self.vox(self.points, self.offsets, boundary=self.boundary, layout=self.bev_fmt,
                     flags=_lib.BEV_RAW, out=self.bev[: self.B], stream=st)
            if self.two_sided:
                self.vox(self.points, self.offsets, boundary=self.boundary_back,
                         layout=self.bev_fmt, flags=_lib.BEV_RAW | _lib.BEV_FLIP_HW,
                         out=self.bev[self.B:], stream=st)
            if bev_done is not None:
                bev_done.record(torch.cuda.current_stream(self.dev))
        if self.infer_graph is not None and not _eager:
            self.infer_graph.replay()
            return self.dets
        return self._infer(st)

    def _infer(self, st):
        if self.with_bev:
            self.engine.forward_into(self.bev, self.outs, self.in_fmt, self.ws, st)
        else:
            self.engine.forward_into(self.x, self.outs, _lib.IN_NCHW3, self.ws, st)
        o = self.outs
        _decoder(o["hm_cen"], o["cen_offset"], o["direction"], o["z_coor"], o["dim"], K=self.K,
                 apply_sigmoid=True, out=self.dets, stream=st, workspace=self.dec_ws)
        return self.dets

    def capture(self):
        """Capture run() into a HIP graph (launch-overhead amortisation)."""
        with torch.cuda.device(self.dev):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self.run(_eager=True)  # warm (module load, lazy init) outside capture
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.run(_eager=True)  # the kernels themselves, never a nested graph launch
            self.graph = g
        return g

    def capture_infer(self):
        """Capture the forward + decode (everything after the BEV) into a HIP graph that run()
        replays: the voxeliser's launches depend on the batch's host frame offsets (a new
        ragged batch per step when streaming), the rest of the step does not."""
        with torch.cuda.device(self.dev):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._infer(_lib.stream_ptr(self.dev))  # warm outside capture
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._infer(_lib.stream_ptr(self.dev))
            self.infer_graph = g
        return g

    def replay(self):
        if self.graph is None:
            return self.run()
        self.graph.replay()
        return self.dets


# ------------------------------------------------------------------ fusion
def iou_matrix(boxes_a, boxes_b, device=None) -> torch.Tensor:
    """calculate_iou for every pair (test6.py:76-101): int [x, y, w, h] boxes -> (na, nb) f64."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    a = torch.as_tensor(np.asarray(boxes_a, np.int32).reshape(-1, 4)).to(dev)
    b = torch.as_tensor(np.asarray(boxes_b, np.int32).reshape(-1, 4)).to(dev)
    out = torch.empty((a.shape[0], b.shape[0]), dtype=torch.float64, device=dev)
    check(lib().sfa_iou_matrix(a.data_ptr() if a.numel() else None, a.shape[0],
                               b.data_ptr() if b.numel() else None, b.shape[0],
                               out.data_ptr() if out.numel() else None, _lib.stream_ptr(dev)),
          "sfa_iou_matrix")
    return out


def gaussian_nms_(boxes: torch.Tensor, conf: torch.Tensor, starts: torch.Tensor, counts: torch.Tensor,
                  sigma: float = 0.5, stream: int = None) -> torch.Tensor:
    """Gaussian soft-NMS in place on device arrays (README.md:250-261 gaussian_nms, batched):
    boxes int32 (N, 4) [x, y, w, h], conf f64 (N,), frame b = the counts[b] entries from
    starts[b] (int32 device tensors). Returns conf."""
    for t, name, dt in ((boxes, "boxes", torch.int32), (conf, "conf", torch.float64),
                        (starts, "starts", torch.int32), (counts, "counts", torch.int32)):
        _require_gpu_tensor(t, "gaussian_nms " + name, dt)
        if not t.is_contiguous():
            raise ValueError(f"gaussian_nms: {name} must be contiguous (updated in place)")
    if starts.numel() != counts.numel():
        raise ValueError("gaussian_nms: starts and counts differ in length")
    st = stream if stream is not None else _lib.stream_ptr(conf.device)
    check(lib().sfa_gaussian_nms(int(starts.numel()), boxes.data_ptr() if boxes.numel() else None,
                                 conf.data_ptr() if conf.numel() else None, starts.data_ptr(),
                                 counts.data_ptr(), float(sigma), st), "sfa_gaussian_nms")
    return conf


def gaussian_nms_frames(frames, sigma: float = 0.5, device=None):
    """[(boxes (n, 4) int, conf (n,) f64), ...] -> the decayed confidences per frame (host f64),
    all frames in one launch."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    counts = np.array([len(c) for _, c in frames], np.int32)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32) if len(frames) else np.zeros(0, np.int32)
    boxes = np.concatenate([np.asarray(b, np.int32).reshape(-1, 4) for b, _ in frames]) if len(frames) \
        else np.zeros((0, 4), np.int32)
    conf = np.concatenate([np.asarray(c, np.float64).reshape(-1) for _, c in frames]) if len(frames) \
        else np.zeros(0, np.float64)
    tb = torch.from_numpy(np.ascontiguousarray(boxes)).to(dev)
    tc = torch.from_numpy(np.ascontiguousarray(conf)).to(dev)
    gaussian_nms_(tb, tc, torch.from_numpy(starts).to(dev), torch.from_numpy(counts).to(dev), sigma)
    out = tc.cpu().numpy()
    return [out[s:s + n] for s, n in zip(starts, counts)]


class FusionResult:
    """Per-frame fused lists (reference order) and NMS survivors (host arrays)."""

    def __init__(self, boxes, conf, cls, src, origin, match, keep):
        self.boxes, self.conf, self.cls, self.src, self.keep = boxes, conf, cls, src, keep
        self.origin, self.match = origin, match


def fuse_frames(frames, conf_threshold=0.3, fusion_iou_threshold=0.7, nms_threshold=0.5,
                mode=_lib.FUSE_BAYES, apply_nms=True, device=None):
    """frames: list of (yolo_boxes (n,4) int, yolo_conf (n,) f64, yolo_cls (n,) int,
    sfa_boxes (m,4) int, sfa_conf (m,) f64).  Runs sfa_fuse_detections on the GPU."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    B = len(frames)
    if B == 0:
        return []
    yb, yc, yk, sb, sc = [], [], [], [], []
    yoff, soff = [0], [0]
    for f in frames:
        a, c, k, s, d = (np.asarray(v) for v in f)
        yb.append(a.astype(np.int32).reshape(-1, 4))
        yc.append(c.astype(np.float64).reshape(-1))
        yk.append(k.astype(np.int32).reshape(-1))
        sb.append(s.astype(np.int32).reshape(-1, 4))
        sc.append(d.astype(np.float64).reshape(-1))
        if yb[-1].shape[0] > 512 or sb[-1].shape[0] > 512:
            raise ValueError("fusion: at most 512 boxes per side per frame")
        yoff.append(yoff[-1] + yb[-1].shape[0])
        soff.append(soff[-1] + sb[-1].shape[0])
    t = lambda x, dt: torch.from_numpy(np.ascontiguousarray(np.concatenate(x) if x else x, dt)).to(dev)
    Y, YC, YK = t(yb, np.int32), t(yc, np.float64), t(yk, np.int32)
    S, SC = t(sb, np.int32), t(sc, np.float64)
    YO = torch.tensor(yoff, dtype=torch.int32, device=dev)
    SO = torch.tensor(soff, dtype=torch.int32, device=dev)
    cap = max(1, yoff[-1] + soff[-1])
    ob = torch.zeros((cap, 4), dtype=torch.int32, device=dev)
    oc = torch.zeros(cap, dtype=torch.float64, device=dev)
    ok = torch.zeros(cap, dtype=torch.int32, device=dev)
    osrc = torch.zeros(cap, dtype=torch.int32, device=dev)
    oorig = torch.zeros(cap, dtype=torch.int32, device=dev)
    omatch = torch.zeros(cap, dtype=torch.int32, device=dev)
    ocount = torch.zeros(B, dtype=torch.int32, device=dev)
    okeep = torch.zeros(cap, dtype=torch.int32, device=dev)
    okc = torch.zeros(B, dtype=torch.int32, device=dev)
    prm = _lib.SfaFusionParams(float(conf_threshold), float(fusion_iou_threshold),
                               float(nms_threshold), int(mode), 1 if apply_nms else 0)
    ptr = lambda x: x.data_ptr() if x.numel() else None
    check(lib().sfa_fuse_detections(B, ptr(Y), ptr(YC), ptr(YK), YO.data_ptr(), ptr(S), ptr(SC),
                                    SO.data_ptr(), ctypes.byref(prm), ob.data_ptr(), oc.data_ptr(),
                                    ok.data_ptr(), osrc.data_ptr(), oorig.data_ptr(),
                                    omatch.data_ptr(), ocount.data_ptr(),
                                    okeep.data_ptr(), okc.data_ptr(), _lib.stream_ptr(dev)),
          "sfa_fuse_detections")
    ob, oc, ok, osrc = ob.cpu().numpy(), oc.cpu().numpy(), ok.cpu().numpy(), osrc.cpu().numpy()
    oorig, omatch = oorig.cpu().numpy(), omatch.cpu().numpy()
    ocount, okeep, okc = ocount.cpu().numpy(), okeep.cpu().numpy(), okc.cpu().numpy()
    out = []
    for b in range(B):
        base, n = yoff[b] + soff[b], int(ocount[b])
        sl = slice(base, base + n)
        keep = okeep[base: base + int(okc[b])].copy() if apply_nms else None
        if n < 0:
            raise ValueError(f"fusion: frame {b} exceeds 512 boxes per side")
        out.append(FusionResult(ob[sl].copy(), oc[sl].copy(), ok[sl].copy(), osrc[sl].copy(),
                                oorig[sl].copy(), omatch[sl].copy(), keep))
    return out


# ------------------------------------------------- post-processing on device
def make_calib(V2C, R0, P2, img_shape) -> "_lib.SfaCalib":
    """One frame's calibration (kitti_data_utils.py:127-139 Calibration fields: V2C 3x4,
    R0 3x3, P2 3x4 — f32 in the reference, widened exactly) + image shape (rows, cols)."""
    c = _lib.SfaCalib()
    c.V2C[:] = [float(v) for v in np.asarray(V2C, np.float64).reshape(-1)[:12]]
    c.R0[:] = [float(v) for v in np.asarray(R0, np.float64)[:3, :3].reshape(-1)]
    c.P2[:] = [float(v) for v in np.asarray(P2, np.float64).reshape(-1)[:12]]
    c.img_h, c.img_w = int(img_shape[0]), int(img_shape[1])
    return c


def calib_tensor(calibs, device) -> torch.Tensor:
    """list of SfaCalib -> device bytes (the C struct array)."""
    arr = (_lib.SfaCalib * len(calibs))(*calibs)
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return host.to(device)


def post_params(num_classes=3, down_ratio=4, peak_thresh=0.2, arith=_lib.REAL_F32,
                boundary=DEFAULT_BOUNDARY, bev_hw=(608, 608)) -> "_lib.SfaPostParams":
    p = _lib.SfaPostParams()
    p.num_classes, p.down_ratio, p.peak_thresh = int(num_classes), int(down_ratio), float(peak_thresh)
    p.bev_h, p.bev_w = int(bev_hw[0]), int(bev_hw[1])
    p.bound_x = float(boundary["maxX"] - boundary["minX"])
    p.bound_y = float(boundary["maxY"] - boundary["minY"])
    p.min_x, p.min_y, p.min_z = (float(boundary[k]) for k in ("minX", "minY", "minZ"))
    p.arith = int(arith)
    return p


def post_process(dets: torch.Tensor, num_classes=3, down_ratio=4, peak_thresh=0.2,
                 arith=_lib.REAL_F32, boundary=DEFAULT_BOUNDARY, bev_hw=(608, 608), out=None):
    """post_processing (evaluation_utils.py:112-163, every frame) + convert_det_to_real_values
    (:177-193) on the GPU.  dets (B, K, 10) f32 -> (preds (B*K, 8) f32, real (B*K, 8) f64,
    offsets (B+1,) int32), all device tensors; frame b owns rows offsets[b]:offsets[b+1]."""
    dets = _require_gpu_tensor(dets, "post_process")
    B, K = int(dets.shape[0]), int(dets.shape[1])
    if dets.dim() != 3 or dets.shape[2] != 10:
        raise ValueError("post_process: dets must be (B, K, 10)")
    dev = dets.device
    if out is None:
        out = (torch.empty((max(1, B * K), 8), dtype=torch.float32, device=dev),
               torch.empty((max(1, B * K), 8), dtype=torch.float64, device=dev),
               torch.empty(B + 1, dtype=torch.int32, device=dev))
    preds, real, off = out
    prm = post_params(num_classes, down_ratio, peak_thresh, arith, boundary, bev_hw)
    check(lib().sfa_post_process(dets.data_ptr(), B, K, ctypes.byref(prm), preds.data_ptr(),
                                 real.data_ptr(), off.data_ptr(), _lib.stream_ptr(dev)),
          "sfa_post_process")
    return preds, real, off


def project_boxes(real: torch.Tensor, offsets: torch.Tensor, calibs, preds=None, conf_min=0.3,
                  conf_source=_lib.CONF_CLASS_ID, extents=False, out=None):
    """convert_sfa3d_to_2d_boxes (test6.py:129-187) on the GPU for every frame.
    calibs: a device tensor from calib_tensor() or a list of SfaCalib (one per frame, or
    one for all).  Returns (boxes (cap, 4) int32, conf f64, row int32, extent f64 or None,
    offsets (B+1,) int32) device tensors (cap = number of real rows)."""
    real = _require_gpu_tensor(real, "project_boxes", torch.float64)
    offsets = _require_gpu_tensor(offsets, "project_boxes offsets", torch.int32)
    dev = real.device
    B = int(offsets.numel()) - 1
    if real.shape[0] == 0:  # no rows: the offsets are all 0, nothing is read
        real = torch.zeros((1, 8), dtype=torch.float64, device=dev)
    if isinstance(calibs, torch.Tensor):
        ct = calibs
        n_cal = ct.numel() // ctypes.sizeof(_lib.SfaCalib)
    else:
        calibs = list(calibs)
        ct, n_cal = calib_tensor(calibs, dev), len(calibs)
    if n_cal not in (1, B) or n_cal == 0:
        raise ValueError("project_boxes: need one calibration or one per frame")
    if conf_source == _lib.CONF_SCORE:
        preds = _require_gpu_tensor(preds, "project_boxes preds")
    cap = max(1, real.shape[0])
    if out is None:
        out = (torch.empty((cap, 4), dtype=torch.int32, device=dev),
               torch.empty(cap, dtype=torch.float64, device=dev),
               torch.empty(cap, dtype=torch.int32, device=dev),
               torch.empty((cap, 4), dtype=torch.float64, device=dev) if extents else None,
               torch.empty(B + 1, dtype=torch.int32, device=dev))
    boxes, conf, row, ext, off = out
    prm = _lib.SfaProjectParams(float(conf_min), int(conf_source), 1 if n_cal == B and B > 1 else 0)
    check(lib().sfa_project_boxes(real.data_ptr(), preds.data_ptr() if preds is not None else None,
                                  offsets.data_ptr(), B, ct.data_ptr(), ctypes.byref(prm),
                                  boxes.data_ptr(), conf.data_ptr(), row.data_ptr(),
                                  ext.data_ptr() if ext is not None else None, off.data_ptr(),
                                  _lib.stream_ptr(dev)),
          "sfa_project_boxes")
    return boxes, conf, row, ext, off


# ------------------------------------------------------- fused LiDAR + camera
class FusionPipeline:
    """BASELINE config #5 on one GPU (test6.py's per-frame flow, batched): sweeps -> BEV ->
    KFPN forward -> decode (DetectorPipeline) -> post_process + convert_det_to_real_values
    (sfa_post_process) -> camera boxes (sfa_project_boxes) -> association, fusion and NMS
    with the camera detector's boxes (sfa_fuse_detections).  Every stage is a HIP kernel on
    device-resident CSR buffers, so run() is one HIP-graph-capturable sequence.

    The camera branch (YOLOv8n, ultralytics) is not part of this framework: its per-frame
    boxes are inputs (``set_camera``), as test6.py:189-209 hands them to the fusion.

    ``nms="gaussian"``: the fused lists get the README's Gaussian soft-NMS (README.md:250-261,
    sfa_gaussian_nms: confidences decayed in place, ``fconf``) instead of the greedy NMS of
    test6.py:104-126 (``fkeep`` then stays unused)."""

    def __init__(self, engine: KfpnEngine, batch: int, calibs, K: int = 50, max_points: int = 0,
                 max_camera_boxes: int = 512, conf_threshold=0.3, fusion_iou_threshold=0.7,
                 nms_threshold=0.5, mode=_lib.FUSE_BAYES, conf_source=_lib.CONF_CLASS_ID,
                 nms: str = "greedy", soft_nms_sigma: float = 0.5):
        self.det = DetectorPipeline(engine, batch, K=K, with_bev=True, max_points=max_points)
        self.B, self.K, self.dev = batch, K, engine.device
        dev = self.dev
        calibs = list(calibs)
        self.calib = calib_tensor(calibs, dev)
        self.conf_source = conf_source
        if nms not in ("greedy", "gaussian"):
            raise ValueError(f"nms must be 'greedy' or 'gaussian', got {nms!r}")
        self.nms, self.soft_nms_sigma = nms, float(soft_nms_sigma)
        self.params = _lib.SfaFusionParams(float(conf_threshold), float(fusion_iou_threshold),
                                           float(nms_threshold), int(mode), 1 if nms == "greedy" else 0)
        self.proj_params = _lib.SfaProjectParams(0.3, int(conf_source),
                                                 1 if len(calibs) == batch and batch > 1 else 0)
        self.post_prm = post_params()
        n = batch * K
        f32, f64, i32 = torch.float32, torch.float64, torch.int32
        with torch.cuda.device(dev):
            self.preds = torch.empty((n, 8), dtype=f32, device=dev)
            self.real = torch.empty((n, 8), dtype=f64, device=dev)
            self.real_off = torch.zeros(batch + 1, dtype=i32, device=dev)
            self.sboxes = torch.empty((n, 4), dtype=i32, device=dev)
            self.sconf = torch.empty(n, dtype=f64, device=dev)
            self.srow = torch.empty(n, dtype=i32, device=dev)
            self.soff = torch.zeros(batch + 1, dtype=i32, device=dev)
            cy = batch * max_camera_boxes
            self.ybox = torch.zeros((cy, 4), dtype=i32, device=dev)
            self.yconf = torch.zeros(cy, dtype=f64, device=dev)
            self.ycls = torch.zeros(cy, dtype=i32, device=dev)
            self.yoff = torch.zeros(batch + 1, dtype=i32, device=dev)
            cap = cy + n
            self.fbox = torch.empty((cap, 4), dtype=i32, device=dev)
            self.fconf = torch.empty(cap, dtype=f64, device=dev)
            self.fcls = torch.empty(cap, dtype=i32, device=dev)
            self.fsrc = torch.empty(cap, dtype=i32, device=dev)
            self.fcount = torch.empty(batch, dtype=i32, device=dev)
            self.fkeep = torch.empty(cap, dtype=i32, device=dev)
            self.fkeep_count = torch.empty(batch, dtype=i32, device=dev)
            self.fstart = torch.zeros(batch, dtype=i32, device=dev)  # frame b's fused list start
        self.max_camera_boxes = max_camera_boxes
        self.graph = None

    def set_points(self, clouds):
        self.det.set_points(clouds)

    def set_camera(self, frames):
        """frames: per frame (boxes (n, 4) int [x, y, w, h], conf (n,), class ids (n,))."""
        if len(frames) != self.B:
            raise ValueError("one camera detection list per frame")
        b, c, k, off = [], [], [], [0]
        for boxes, conf, cls in frames:
            boxes = np.asarray(boxes, np.int32).reshape(-1, 4)
            if boxes.shape[0] > min(512, self.max_camera_boxes):
                raise ValueError("at most 512 camera boxes per frame")
            b.append(boxes)
            c.append(np.asarray(conf, np.float64).reshape(-1))
            k.append(np.asarray(cls, np.int32).reshape(-1))
            off.append(off[-1] + boxes.shape[0])
        n = off[-1]
        if n:
            self.ybox[:n].copy_(torch.from_numpy(np.concatenate(b)))
            self.yconf[:n].copy_(torch.from_numpy(np.concatenate(c)))
            self.ycls[:n].copy_(torch.from_numpy(np.concatenate(k)))
        self.yoff.copy_(torch.tensor(off, dtype=torch.int32))

    def run(self):
        st = _lib.stream_ptr(self.dev)
        L = lib()
        dets = self.det.run()
        check(L.sfa_post_process(dets.data_ptr(), self.B, self.K, ctypes.byref(self.post_prm),
                                 self.preds.data_ptr(), self.real.data_ptr(),
                                 self.real_off.data_ptr(), st), "sfa_post_process")
        check(L.sfa_project_boxes(self.real.data_ptr(), self.preds.data_ptr(),
                                  self.real_off.data_ptr(), self.B, self.calib.data_ptr(),
                                  ctypes.byref(self.proj_params), self.sboxes.data_ptr(),
                                  self.sconf.data_ptr(), self.srow.data_ptr(), None,
                                  self.soff.data_ptr(), st), "sfa_project_boxes")
        check(L.sfa_fuse_detections(self.B, self.ybox.data_ptr(), self.yconf.data_ptr(),
                                    self.ycls.data_ptr(), self.yoff.data_ptr(),
                                    self.sboxes.data_ptr(), self.sconf.data_ptr(),
                                    self.soff.data_ptr(), ctypes.byref(self.params),
                                    self.fbox.data_ptr(), self.fconf.data_ptr(),
                                    self.fcls.data_ptr(), self.fsrc.data_ptr(), None, None,
                                    self.fcount.data_ptr(), self.fkeep.data_ptr(),
                                    self.fkeep_count.data_ptr(), st), "sfa_fuse_detections")
        if self.nms == "gaussian":
            torch.add(self.yoff[:-1], self.soff[:-1], out=self.fstart)  # on the current stream (= st)
            check(L.sfa_gaussian_nms(self.B, self.fbox.data_ptr(), self.fconf.data_ptr(), self.fstart.data_ptr(),
                                     self.fcount.data_ptr(), self.soft_nms_sigma, st), "sfa_gaussian_nms")
        return self.fcount

    def capture(self):
        with torch.cuda.device(self.dev):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self.run()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.run()
            self.graph = g
        return g

    def replay(self):
        if self.graph is None:
            return self.run()
        self.graph.replay()
        return self.fcount

    def results(self):
        """Host copy per frame: (fused boxes, conf, cls, source, NMS keep indices); with
        nms="gaussian" conf is the decayed confidence and keep is every index (nothing dropped)."""
        yoff = self.yoff.cpu().numpy()
        soff = self.soff.cpu().numpy()
        cnt, kc = self.fcount.cpu().numpy(), self.fkeep_count.cpu().numpy()
        fb, fc, fk, fs, keep = (t.cpu().numpy() for t in (self.fbox, self.fconf, self.fcls,
                                                          self.fsrc, self.fkeep))
        out = []
        for b in range(self.B):
            base = yoff[b] + soff[b]
            n = int(cnt[b])
            kp = np.arange(max(n, 0), dtype=keep.dtype) if self.nms == "gaussian" else keep[base:base + int(kc[b])]
            out.append((fb[base:base + n], fc[base:base + n], fk[base:base + n], fs[base:base + n], kp))
        return out
