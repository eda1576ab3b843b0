"""C-ABI checks that need no GPU: the library loads, exports every symbol the
public header declares, enumerates the reference state_dict layout, packs
weights (BatchNorm folding + OHWI re-layout) and reports errors by code."""
import ctypes
import os
import re

import numpy as np
import pytest

import golden_cases as gc
from conftest import REPO
from sfa_hip import _lib
from sfa_hip.runtime import pack_state_dict

HEADER = os.path.join(REPO, "include", "sfa_hip.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sfa_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(L, s), f"{s} declared in include/sfa_hip.h but not exported"
    assert sorted(_lib.EXPORTED_SYMBOLS) == syms, "ctypes prototypes out of sync with the header"
    assert L.sfa_abi_version() == _lib.ABI_VERSION == 2


def test_exported_symbols_are_only_the_abi():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True).stdout
    text_syms = sorted(l.split()[-1] for l in out.splitlines() if " T " in l)
    assert text_syms == header_symbols()


def test_state_layout_matches_reference(golden):
    arch = _lib.make_arch(gc.HEADS)
    layout = _lib.state_layout(arch)
    assert [n for n, _ in layout] == [str(n) for n in golden.model["state_names"]]
    assert [s for _, s in layout] == [s for _, s in gc.state_spec(golden.model)]


def _unpack_plan_offsets(arch):
    """Recompute the packed layout independently (mirror of model.hip make_plan)."""
    cur = 0
    out = {}

    def take(n):
        nonlocal cur
        o = cur
        cur = (cur + n + 15) // 16 * 16
        return o

    def conv(key, N, K):
        Kp = (K + 15) // 16 * 16
        out[key] = (take(N * Kp), take(N), N, Kp)
        out[key + "/wx"] = take((3 * N * Kp + 1) // 2)  # bf16x6 terms [3][N][Kpad]
        out[key + "/wh"] = take(N * Kp)                 # fp16x3 terms [2][N][Kpad]
        out[key + "/winv"] = take(N)

    conv("stem", 64, 196)
    inpl = 64
    for li in range(4):
        planes = 64 << li
        for bi in range(2):
            cin = inpl if bi == 0 else planes
            ds = bi == 0 and li > 0
            conv(f"l{li}b{bi}c1", planes, 9 * cin)
            conv(f"l{li}b{bi}c2", planes, 9 * planes + (inpl if ds else 0))
        inpl = planes
    for i, (n, k) in enumerate(((256, 768), (128, 384), (64, 192))):
        conv(f"fpn{i}", n, k)
    return out, cur


def test_pack_weights_folds_batchnorm(golden):
    arch = _lib.make_arch(gc.HEADS)
    sd = gc.state_dict_np(golden.model)
    packed = pack_state_dict(sd, arch)
    assert packed.size == _lib.lib().sfa_packed_floats(ctypes.byref(arch))
    offs, _ = _unpack_plan_offsets(arch)
    # stem: W[o][(kh*7+kw)*4 + c] = w[o,c,kh,kw] * g/sqrt(v+eps); channel 3 and K pad are 0
    w_off, b_off, N, Kp = offs["stem"]
    W = packed[w_off:w_off + N * Kp].reshape(N, Kp)
    scale = sd["bn1.weight"].astype(np.float64) / np.sqrt(sd["bn1.running_var"].astype(np.float64) + 1e-5)
    exp = (sd["conv1.weight"].astype(np.float64) * scale[:, None, None, None]).astype(np.float32)
    got = W[:, :196].reshape(64, 7, 7, 4)
    np.testing.assert_array_equal(got[..., :3], exp.transpose(0, 2, 3, 1))
    assert np.all(got[..., 3] == 0) and np.all(W[:, 196:] == 0)
    shift = sd["bn1.bias"] - sd["bn1.running_mean"] * scale
    np.testing.assert_allclose(packed[b_off:b_off + 64], shift, rtol=1e-6, atol=1e-7)
    # layer2.0.conv2 + fused downsample: K = 9*128 + 64, bias = shift2 + shift_ds
    w_off, b_off, N, Kp = offs["l1b0c2"]
    W = packed[w_off:w_off + N * Kp].reshape(N, Kp)
    p = "layer2.0."
    s2 = sd[p + "bn2.weight"] / np.sqrt(sd[p + "bn2.running_var"].astype(np.float64) + 1e-5)
    sds = sd[p + "downsample.1.weight"] / np.sqrt(sd[p + "downsample.1.running_var"].astype(np.float64) + 1e-5)
    np.testing.assert_allclose(W[:, 1152:], sd[p + "downsample.0.weight"][:, :, 0, 0] * sds[:, None],
                               rtol=1e-6)
    np.testing.assert_allclose(W[:, :1152].reshape(128, 3, 3, 128),
                               (sd[p + "conv2.weight"] * s2[:, None, None, None]).transpose(0, 2, 3, 1),
                               rtol=1e-6)
    b_exp = (sd[p + "bn2.bias"] - sd[p + "bn2.running_mean"] * s2) + (
        sd[p + "downsample.1.bias"] - sd[p + "downsample.1.running_mean"] * sds)
    np.testing.assert_allclose(packed[b_off:b_off + 128], b_exp, rtol=1e-5, atol=1e-7)
    # FPN conv_up_level1: no BN, K order = [upsampled layer4 (512) | layer3 (256)]
    w_off, b_off, N, Kp = offs["fpn0"]
    np.testing.assert_array_equal(packed[w_off:w_off + N * Kp].reshape(N, Kp),
                                  sd["conv_up_level1.weight"][:, :, 0, 0])
    # bf16x6 terms: three bf16 values (round to nearest even) summing exactly to W
    for key in ("stem", "l1b0c2", "l3b1c2", "fpn0"):
        w_off, _, N, Kp = offs[key]
        W = packed[w_off:w_off + N * Kp]
        x = offs[key + "/wx"]
        t = packed[x:x + (3 * N * Kp + 1) // 2].view(np.uint16)[:3 * N * Kp].reshape(3, -1)
        f = (t.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
        np.testing.assert_array_equal(f.sum(0), W.astype(np.float64))
        assert np.all(np.abs(f[1]) <= np.abs(f[0]) * 2.0 ** -8 + 1e-45)
        hi = (W.view(np.uint32) + 0x7FFF + ((W.view(np.uint32) >> 16) & 1)) >> 16
        np.testing.assert_array_equal(t[0], hi.astype(np.uint16))
        # fp16x3: W[n] * 2^(13 - e[n]) = hi + lo (fp16, round to nearest even), winv = 2^(e - 13)
        Wn = W.reshape(N, Kp)
        winv = packed[offs[key + "/winv"]:offs[key + "/winv"] + N]
        e = np.floor(np.log2(np.abs(Wn).max(1)))
        np.testing.assert_array_equal(winv, np.exp2(e - 13).astype(np.float32))
        x2 = offs[key + "/wh"]
        hl = packed[x2:x2 + N * Kp].view(np.float16).reshape(2, N, Kp)
        scaled = Wn * (1.0 / winv[:, None])
        assert np.abs(scaled).max() < 2.0 ** 14
        np.testing.assert_array_equal(hl[0], scaled.astype(np.float16))
        np.testing.assert_array_equal(hl[1], (scaled - hl[0].astype(np.float32)).astype(np.float16))
        rel = np.abs(hl[0].astype(np.float64) + hl[1] - scaled) / np.abs(scaled).max(1, keepdims=True)
        assert rel.max() <= 2.0 ** -22  # 22 significand bits


def test_pack_rejects_wrong_state():
    arch = _lib.make_arch(gc.HEADS)
    with pytest.raises(KeyError):
        pack_state_dict({}, arch)
    L = _lib.lib()
    junk = np.zeros(10, np.float32)
    out = np.zeros(10, np.float32)
    rc = L.sfa_pack_weights(ctypes.byref(arch), junk.ctypes.data, 10, out.ctypes.data)
    assert rc == -1 and b"state floats" in L.sfa_last_error_string()


def test_unsupported_arch_reports_error():
    L = _lib.lib()
    arch = _lib.make_arch(gc.HEADS, num_layers=34)
    assert L.sfa_state_count(ctypes.byref(arch)) == -1
    assert b"fpn_resnet_18" in L.sfa_last_error_string()
    arch = _lib.make_arch(gc.HEADS, head_conv=32)
    assert L.sfa_packed_floats(ctypes.byref(arch)) == 0


def test_argument_errors_before_any_launch():
    """Shape/argument validation runs on the host and never touches the device."""
    L = _lib.lib()
    assert L.sfa_decode(None, None, None, None, None, 1, 3, 152, 152, 50, 1, None, None, 0, None) == -1
    ws = ctypes.create_string_buffer(16)
    p = ctypes.cast(ws, ctypes.c_void_p)
    # K > 256
    assert L.sfa_decode(p, p, p, p, p, 1, 3, 152, 152, 300, 1, p, p, 16, None) == -1
    assert b"K" in L.sfa_last_error_string()
    # H*W too large for the LDS-resident peak map
    assert L.sfa_decode(p, p, p, p, p, 1, 3, 304, 304, 50, 1, p, p, 16, None) == -1
    offs = (ctypes.c_int64 * 2)(0, 10)
    bnd = (ctypes.c_double * 6)(0, 50, -25, 25, -2.73, 1.27)
    big = L.sfa_bev_scratch_size(1)
    assert L.sfa_bev_voxelize(p, offs, 0, bnd, 0, 2, p, p, big, None) == -1
    assert L.sfa_bev_voxelize(p, offs, 1, bnd, 32, 2, p, p, big, None) == -1  # unknown flag bit
    # a scratch smaller than the batch's layout is refused before any launch (SFA_E_WORKSPACE)
    assert L.sfa_bev_voxelize(p, offs, 1, bnd, 0, 2, p, p, big - 1, None) == -4
    assert b"scratch" in L.sfa_last_error_string()
    assert L.sfa_bev_scratch_size(16) == 2 * 16 * 608 * 608 * 12  # atomic-path cells + binned records
    # kernel probe (bench roofline): null model / unknown flags / reading a disabled probe
    ms = (ctypes.c_float * 3)()
    assert L.sfa_model_set_probe(None, _lib.PROBE_SERIAL) == -1
    assert L.sfa_model_probe_times(None, ms, 3) == -1
    arch = _lib.make_arch(gc.HEADS)
    h = ctypes.c_void_p()
    assert L.sfa_model_create(ctypes.byref(arch), p, ctypes.byref(h)) == 0
    try:
        assert L.sfa_model_set_probe(h, 8) == -1 and b"flags" in L.sfa_last_error_string()
        assert L.sfa_model_set_probe(h, _lib.PROBE_SERIAL) == 0  # no events needed
        assert L.sfa_model_probe_times(h, ms, 3) == -1 and b"not enabled" in L.sfa_last_error_string()
        assert L.sfa_model_probe_times(h, ms, 4) == -1
        # kernel-choice options live in the handle (no env reads on the launch path)
        v = ctypes.c_int()
        defaults = {_lib.OPT_STEM_PATCH: 1, _lib.OPT_FPN_COMMUTE: 7, _lib.OPT_FPN_GEMM: 61,
                    _lib.OPT_SPLITK_TICKETS: 1}
        assert len(defaults) == _lib.OPT_COUNT
        for key, val in defaults.items():
            assert L.sfa_model_get_option(h, key, ctypes.byref(v)) == 0 and v.value == val, key
        for form in (0, 1):  # implicit-GEMM + max-pool / patch stem + merge
            assert L.sfa_model_set_option(h, _lib.OPT_STEM_PATCH, form) == 0
            assert L.sfa_model_get_option(h, _lib.OPT_STEM_PATCH, ctypes.byref(v)) == 0 and v.value == form
        assert L.sfa_model_set_option(h, _lib.OPT_STEM_PATCH, 2) == -1
        assert L.sfa_model_set_option(h, _lib.OPT_FPN_COMMUTE, 9) == -1
        assert L.sfa_model_set_option(h, _lib.OPT_FPN_COMMUTE, 5) == 0
        assert L.sfa_model_set_option(h, _lib.OPT_FPN_GEMM, 64) == -1
        assert L.sfa_model_set_option(h, _lib.OPT_FPN_GEMM, 63) == 0
        assert L.sfa_model_set_option(h, _lib.OPT_SPLITK_TICKETS, 2) == -1
        assert L.sfa_model_set_option(h, _lib.OPT_SPLITK_TICKETS, 0) == 0
        # the round-3 A/B keys (tune bits, grouped heads, ...) are gone: unknown keys now
        for gone in range(_lib.OPT_COUNT, 8):
            assert L.sfa_model_set_option(h, gone, 0) == -1
        assert L.sfa_model_set_option(h, 99, 0) == -1 and b"unknown key" in L.sfa_last_error_string()
        assert L.sfa_model_get_option(h, 99, ctypes.byref(v)) == -1
        assert L.sfa_model_set_option(None, 0, 0) == -1
    finally:
        L.sfa_model_destroy(h)


def test_workspace_sizes():
    L = _lib.lib()
    assert L.sfa_decode_workspace_size(16, 3, 50) >= 16 * 3 * 50 * 8
    assert L.sfa_filter_scratch_size(132880) >= 4 * ((132880 + 2047) // 2048)


def test_forward_batch_limit():
    """include/sfa_hip.h batch limit: one pass holds floor((2^31 - 1) / (32 H W)) frames (the conv
    kernels' 32-bit buffer offsets; up_level3 is the widest conv input), 181 at 608 x 608; the
    workspace is sized for one pass; a frame too large for any pass is refused before a launch."""
    L = _lib.lib()
    assert L.sfa_forward_max_batch(608, 608) == 181
    assert L.sfa_forward_max_batch(608, 608) == ((1 << 31) - 1) // (32 * 608 * 608)
    assert L.sfa_forward_max_batch(96, 96) == ((1 << 31) - 1) // (32 * 96 * 96)
    assert L.sfa_forward_max_batch(8192, 8192) == 0 and L.sfa_forward_max_batch(0, 608) == 0
    arch = _lib.make_arch(gc.HEADS)
    ws = ctypes.create_string_buffer(16)
    p = ctypes.cast(ws, ctypes.c_void_p)
    h = ctypes.c_void_p()
    assert L.sfa_model_create(ctypes.byref(arch), p, ctypes.byref(h)) == 0
    try:
        one = L.sfa_forward_workspace_size(h, 181, 608, 608)
        assert one > 0 and L.sfa_forward_workspace_size(h, 182, 608, 608) == one
        assert L.sfa_forward_workspace_size(h, 1000, 608, 608) == one
        assert L.sfa_forward_workspace_size(h, 180, 608, 608) < one
        assert L.sfa_forward_workspace_size(h, 1, 8192, 8192) == 0
        assert L.sfa_forward_buffer_offset(h, 1000, 608, 608, 0) == L.sfa_forward_buffer_offset(h, 181, 608, 608, 0)
        outs = (ctypes.c_void_p * arch.num_heads)(*([p.value] * arch.num_heads))
        # H = W = 8192: one frame's up_level3 alone is 2 GiB -> SFA_E_UNSUPPORTED, no launch
        assert L.sfa_model_forward(h, p, _lib.IN_NCHW3, 1, 8192, 8192, outs, p, 1 << 40, None) == -2
        assert b"32-bit buffer offsets" in L.sfa_last_error_string()
        # a workspace sized for fewer frames than one pass is refused (SFA_E_WORKSPACE)
        assert L.sfa_model_forward(h, p, _lib.IN_NCHW3, 200, 608, 608, outs, p, one - 1, None) == -4
    finally:
        L.sfa_model_destroy(h)
