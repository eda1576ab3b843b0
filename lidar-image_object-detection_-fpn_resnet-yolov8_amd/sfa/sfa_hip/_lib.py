"""ctypes binding of libsfa_hip.so (the C ABI declared in include/sfa_hip.h).

The library is the product: there is no CPU fallback.  If the shared object is
missing or fails to load, every entry point raises ``SfaNativeError`` — the
drop-in modules never substitute a Python/torch computation.

torch is imported first so that the process' HIP runtime is torch's
(libamdhip64.so.7 — same SONAME as /opt/rocm's); the library then binds to it
and device pointers / streams from torch are valid on its side.
"""

from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before ours)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SFA_HIP_LIB", os.path.join(_HERE, "libsfa_hip.so"))

SFA_OK = 0
ABI_VERSION = 2  # include/sfa_hip.h SFA_ABI_VERSION
SFA_MAX_HEADS = 8
SFA_BEV_MAX_BATCH = 64
BEV_NCHW3_F32, BEV_NCHW3_F64, BEV_NHWC4_F32 = 0, 1, 2
BEV_RAW, BEV_PREFILTERED, BEV_FLIP_HW, BEV_FORCE_ATOMIC, BEV_FORCE_BINNED, BEV_STRIP8 = 0, 1, 2, 4, 8, 16
# sfa_model_set_option keys (include/sfa_hip.h sfa_model_option)
OPT_STEM_PATCH, OPT_FPN_COMMUTE, OPT_FPN_GEMM, OPT_SPLITK_TICKETS = 0, 1, 2, 3
OPT_COUNT = 4  # keys 0 .. OPT_COUNT - 1
IN_NCHW3, IN_NHWC4, IN_NCHW3_FLIP_HW = 0, 1, 2


class SfaNativeError(RuntimeError):
    """Raised when the HIP library is unavailable or returns an error."""


class SfaArch(ctypes.Structure):
    _fields_ = [
        ("num_layers", ctypes.c_int),
        ("head_conv", ctypes.c_int),
        ("num_heads", ctypes.c_int),
        ("head_channels", ctypes.c_int * SFA_MAX_HEADS),
        ("head_names", (ctypes.c_char * 32) * SFA_MAX_HEADS),
    ]


_c_size = ctypes.c_size_t
_c_int = ctypes.c_int
_c_i64 = ctypes.c_int64
_vp = ctypes.c_void_p
_PROTOS = {
    "sfa_abi_version": (_c_int, []),
    "sfa_last_error_string": (ctypes.c_char_p, []),
    "sfa_bev_scratch_size": (_c_size, [_c_int]),
    "sfa_bev_voxelize": (_c_int, [_vp, ctypes.POINTER(_c_i64), _c_int, ctypes.POINTER(ctypes.c_double),
                                  _c_int, _c_int, _vp, _vp, _c_size, _vp]),
    "sfa_filter_scratch_size": (_c_size, [_c_i64]),
    "sfa_filter_points": (_c_int, [_vp, _c_i64, ctypes.POINTER(ctypes.c_double), _vp, _vp, _vp,
                                   _c_size, _vp]),
    "sfa_state_count": (_c_int, [ctypes.POINTER(SfaArch)]),
    "sfa_state_entry": (_c_int, [ctypes.POINTER(SfaArch), _c_int, ctypes.c_char_p, _c_int,
                                 ctypes.POINTER(_c_i64), ctypes.POINTER(_c_int)]),
    "sfa_state_floats": (_c_size, [ctypes.POINTER(SfaArch)]),
    "sfa_packed_floats": (_c_size, [ctypes.POINTER(SfaArch)]),
    "sfa_pack_weights": (_c_int, [ctypes.POINTER(SfaArch), _vp, _c_size, _vp]),
    "sfa_model_create": (_c_int, [ctypes.POINTER(SfaArch), _vp, ctypes.POINTER(_vp)]),
    "sfa_model_destroy": (None, [_vp]),
    "sfa_forward_max_batch": (_c_int, [_c_int, _c_int]),
    "sfa_forward_workspace_size": (_c_size, [_vp, _c_int, _c_int, _c_int]),
    "sfa_forward_buffer_offset": (_c_i64, [_vp, _c_int, _c_int, _c_int, _c_int]),
    "sfa_model_forward": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int, _c_int, ctypes.POINTER(_vp),
                                   _vp, _c_size, _vp]),
    "sfa_sigmoid_clamp_inplace": (_c_int, [_vp, _c_i64, _vp]),
    "sfa_decode_workspace_size": (_c_size, [_c_int, _c_int, _c_int]),
    "sfa_decode": (_c_int, [_vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                            _vp, _vp, _c_size, _vp]),
}

MATH_F32, MATH_BF16X6, MATH_FP16X3 = 0, 1, 2
_PROTOS["sfa_model_set_math"] = (_c_int, [_vp, _c_int])
_PROTOS["sfa_model_get_math"] = (_c_int, [_vp])
_PROTOS["sfa_model_set_option"] = (_c_int, [_vp, _c_int, _c_int])
_PROTOS["sfa_model_get_option"] = (_c_int, [_vp, _c_int, ctypes.POINTER(_c_int)])
PROBE_HEADS, PROBE_SERIAL = 1, 2
_PROTOS["sfa_model_set_probe"] = (_c_int, [_vp, _c_int])
_PROTOS["sfa_model_set_side_streams"] = (_c_int, [_vp, _c_int])
_PROTOS["sfa_model_probe_times"] = (_c_int, [_vp, ctypes.POINTER(ctypes.c_float), _c_int])
_PROTOS["sfa_heat_nms"] = (_c_int, [_vp, _vp, _c_i64, _c_int, _c_int, _vp])
_PROTOS["sfa_topk_workspace_size"] = (_c_size, [_c_int, _c_int, _c_int])
_PROTOS["sfa_topk"] = (_c_int, [_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp,
                                _vp, _c_size, _vp])
_PROTOS["sfa_gather_feat"] = (_c_int, [_vp, _c_int, _c_i64, _c_int, _c_i64, _c_i64, _c_int, _vp, _c_int, _vp, _vp])


def math_from_env(default=MATH_FP16X3) -> int:
    """SFA_MATH=f32 | bf16x6 | fp16x3 selects the convolution arithmetic (include/sfa_hip.h)."""
    v = os.environ.get("SFA_MATH", "").strip().lower()
    if not v:
        return default
    if v in ("f32", "fp32"):
        return MATH_F32
    if v in ("bf16x6", "x6"):
        return MATH_BF16X6
    if v in ("fp16x3", "h3"):
        return MATH_FP16X3
    raise ValueError(f"SFA_MATH={v!r}: expected 'f32', 'bf16x6' or 'fp16x3'")


class SfaFusionParams(ctypes.Structure):
    _fields_ = [("conf_threshold", ctypes.c_double), ("fusion_iou_threshold", ctypes.c_double),
                ("nms_threshold", ctypes.c_double), ("mode", ctypes.c_int),
                ("apply_nms", ctypes.c_int)]


FUSE_BAYES, FUSE_WEIGHTED = 0, 1
SRC_YOLO, SRC_LIDAR, SRC_FUSED = 0, 1, 2
_PROTOS["sfa_iou_matrix"] = (_c_int, [_vp, _c_int, _vp, _c_int, _vp, _vp])
_PROTOS["sfa_gaussian_nms"] = (_c_int, [_c_int, _vp, _vp, _vp, _vp, ctypes.c_double, _vp])
_PROTOS["sfa_fuse_detections"] = (_c_int, [_c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                           ctypes.POINTER(SfaFusionParams), _vp, _vp, _vp, _vp,
                                           _vp, _vp, _vp, _vp, _vp, _vp])


class SfaPostParams(ctypes.Structure):
    _fields_ = [("num_classes", ctypes.c_int), ("down_ratio", ctypes.c_int),
                ("peak_thresh", ctypes.c_float), ("bev_h", ctypes.c_int), ("bev_w", ctypes.c_int),
                ("bound_x", ctypes.c_double), ("bound_y", ctypes.c_double),
                ("min_x", ctypes.c_double), ("min_y", ctypes.c_double), ("min_z", ctypes.c_double),
                ("arith", ctypes.c_int)]


class SfaCalib(ctypes.Structure):
    _fields_ = [("V2C", ctypes.c_double * 12), ("R0", ctypes.c_double * 9),
                ("P2", ctypes.c_double * 12), ("img_h", ctypes.c_int32), ("img_w", ctypes.c_int32)]


class SfaProjectParams(ctypes.Structure):
    _fields_ = [("conf_min", ctypes.c_double), ("conf_source", ctypes.c_int),
                ("calib_per_frame", ctypes.c_int)]


REAL_F32, REAL_F64 = 0, 1
CONF_CLASS_ID, CONF_SCORE = 0, 1
_PROTOS["sfa_post_process"] = (_c_int, [_vp, _c_int, _c_int, ctypes.POINTER(SfaPostParams), _vp,
                                        _vp, _vp, _vp])
_PROTOS["sfa_project_boxes"] = (_c_int, [_vp, _vp, _vp, _c_int, _vp,
                                         ctypes.POINTER(SfaProjectParams), _vp, _vp, _vp, _vp,
                                         _vp, _vp])
_PROTOS["sfa_bin_stream_create"] = (_c_int, [ctypes.POINTER(ctypes.c_char_p), _c_int, _c_int, _c_i64,
                                             _c_int, _c_int, ctypes.POINTER(_vp)])
_PROTOS["sfa_bin_stream_next"] = (_c_int, [_vp, _vp, _c_i64, ctypes.POINTER(_c_i64),
                                           ctypes.POINTER(_c_int), _vp])
_PROTOS["sfa_bin_stream_destroy"] = (None, [_vp])
EXPORTED_SYMBOLS = tuple(_PROTOS)

_lib = None
_load_error = None


def lib():
    """The loaded library; raises SfaNativeError (never falls back) if unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise SfaNativeError(_load_error)
    if not os.path.isfile(LIB_PATH):
        _load_error = (f"HIP library not built: {LIB_PATH} is missing "
                       "(run __graft_entry__.build() or make -C <pkg>/csrc)")
        raise SfaNativeError(_load_error)
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        _load_error = f"cannot load {LIB_PATH}: {e}"
        raise SfaNativeError(_load_error) from e
    for name, (res, args) in _PROTOS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.sfa_abi_version() != ABI_VERSION:
        raise SfaNativeError("libsfa_hip ABI version mismatch")
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != SFA_OK:
        msg = lib().sfa_last_error_string()
        raise SfaNativeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def make_arch(heads: dict, head_conv: int = 64, num_layers: int = 18) -> SfaArch:
    """heads: {name: channels} in FORWARD (insertion) order (fpn_resnet.py:220)."""
    a = SfaArch()
    a.num_layers = int(num_layers)
    a.head_conv = int(head_conv)
    items = list(heads.items())
    if not 1 <= len(items) <= SFA_MAX_HEADS:
        raise ValueError(f"{len(items)} heads; 1..{SFA_MAX_HEADS} supported")
    a.num_heads = len(items)
    for j, (name, ch) in enumerate(items):
        a.head_channels[j] = int(ch)
        nb = name.encode()
        if len(nb) >= 32:
            raise ValueError(f"head name too long: {name}")
        a.head_names[j].value = nb
    return a


def state_layout(arch: SfaArch):
    """[(name, shape tuple)] of the reference state_dict, from the C side."""
    L = lib()
    n = L.sfa_state_count(ctypes.byref(arch))
    if n < 0:
        check(-1, "sfa_state_count")
    out = []
    buf = ctypes.create_string_buffer(128)
    shape = (_c_i64 * 4)()
    nd = _c_int()
    for i in range(n):
        check(L.sfa_state_entry(ctypes.byref(arch), i, buf, 128, shape, ctypes.byref(nd)),
              "sfa_state_entry")
        out.append((buf.value.decode(), tuple(int(shape[k]) for k in range(nd.value))))
    return out


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
