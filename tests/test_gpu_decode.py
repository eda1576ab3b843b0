"""GPU parity of _sigmoid / decode vs the reference fixtures and the oracle.

Bar (BASELINE north_star): peak indices / top-K selection bit-exact; the HIP
decode on the reference's own sigmoid maps reproduces the reference's (B, K, 10)
detections bit for bit on tie-free inputs.
"""
import numpy as np
import pytest
import torch

import golden_cases as gc
from oracle import decode_oracle
from sfa_hip import runtime

pytestmark = pytest.mark.gpu


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("case", ["b2_152_k50", "b3_64_k40"])
def test_decode_bit_exact_on_reference_maps(golden, gpu, case):
    from utils.evaluation_utils import decode, post_processing, convert_det_to_real_values
    g = golden.decode
    inp = gc.decode_inputs(case)
    dets = decode(_t(g[f"{case}/hm_sigmoid"], gpu), _t(g[f"{case}/off_sigmoid"], gpu),
                  _t(inp["dir"], gpu), _t(inp["z"], gpu), _t(inp["dim"], gpu), K=inp["K"])
    assert dets.device == gpu and dets.dtype == torch.float32
    d = dets.cpu().numpy()
    np.testing.assert_array_equal(d, g[f"{case}/dets"])
    post = post_processing(d.copy(), 3, 4, 0.2)
    for j in range(3):
        np.testing.assert_array_equal(post[0][j], g[f"{case}/post_cls{j}"])
    np.testing.assert_array_equal(convert_det_to_real_values(post[0]), g[f"{case}/real"])


def test_decode_plateaus(golden, gpu):
    g = golden.decode
    case = "b1_32_k20_plateau"
    inp = gc.decode_inputs(case)
    hm, off = g[f"{case}/hm_sigmoid"], g[f"{case}/off_sigmoid"]
    d = runtime.decode(_t(hm, gpu), _t(off, gpu), _t(inp["dir"], gpu), _t(inp["z"], gpu),
                       _t(inp["dim"], gpu), K=inp["K"]).cpu().numpy()
    # our deterministic tie order == the oracle's (lower index, then lower class)
    np.testing.assert_array_equal(d, decode_oracle.decode(hm, off, inp["dir"], inp["z"], inp["dim"],
                                                          K=inp["K"]))
    ref = g[f"{case}/dets"]
    np.testing.assert_array_equal(np.sort(d[0, :, 0]), np.sort(ref[0, :, 0]))


def test_sigmoid_inplace(golden, gpu):
    from utils.torch_utils import _sigmoid
    inp = gc.decode_inputs("b2_152_k50")
    x = _t(inp["hm"], gpu)
    y = _sigmoid(x)
    assert y.data_ptr() == x.data_ptr()
    ref = golden.decode["b2_152_k50/hm_sigmoid"]
    assert np.max(np.abs(y.cpu().numpy() - ref)) <= 2.4e-7  # <= 2 ulp of torch's CPU sigmoid
    sat = _sigmoid(torch.tensor([-50.0, 50.0, 0.0], device=gpu)).cpu().numpy()
    np.testing.assert_array_equal(sat, np.float32([1e-4, 1 - 1e-4, 0.5]))


@pytest.mark.parametrize("case", ["b2_152_k50", "b3_64_k40"])
def test_fused_sigmoid_decode(golden, gpu, case):
    """apply_sigmoid=1 (the bench path) == HIP _sigmoid then decode, bit for bit."""
    inp = gc.decode_inputs(case)
    dev = {k: _t(inp[k], gpu) for k in ("hm", "off", "dir", "z", "dim")}
    fused = runtime.decode(dev["hm"], dev["off"], dev["dir"], dev["z"], dev["dim"], K=inp["K"],
                           apply_sigmoid=True).cpu().numpy()
    hm = runtime.sigmoid_clamp_(dev["hm"].clone())
    off = runtime.sigmoid_clamp_(dev["off"].clone())
    two = runtime.decode(hm, off, dev["dir"], dev["z"], dev["dim"], K=inp["K"]).cpu().numpy()
    np.testing.assert_array_equal(fused, two)
    # and within fp tolerance of the reference (sigmoid ulps only)
    ref = golden.decode[f"{case}/dets"]
    np.testing.assert_array_equal(fused[..., 9], ref[..., 9])
    np.testing.assert_allclose(fused, ref, rtol=0, atol=1e-6)


def test_decode_random_vs_oracle_many(gpu):
    """Random tie-free maps at the production shape, several K."""
    rng = np.random.default_rng(3)
    for B, K in ((16, 50), (4, 1), (2, 256), (1, 100)):
        hm = rng.random((B, 3, 152, 152), dtype=np.float32)
        off = rng.random((B, 2, 152, 152), dtype=np.float32)
        dr = rng.standard_normal((B, 2, 152, 152)).astype(np.float32)
        z = rng.standard_normal((B, 1, 152, 152)).astype(np.float32)
        dm = rng.standard_normal((B, 3, 152, 152)).astype(np.float32)
        got = runtime.decode(_t(hm, gpu), _t(off, gpu), _t(dr, gpu), _t(z, gpu), _t(dm, gpu),
                             K=K).cpu().numpy()
        np.testing.assert_array_equal(got, decode_oracle.decode(hm, off, dr, z, dm, K=K))


def test_decode_all_zero_and_negative_maps(gpu):
    """Degenerate maps: all-equal scores (every pixel a plateau peak) and negatives."""
    B, H, W, K = 2, 40, 48, 30
    z1 = np.zeros((B, 1, H, W), np.float32)
    maps = dict(off=np.zeros((B, 2, H, W), np.float32), dir=np.zeros((B, 2, H, W), np.float32),
                z=z1, dim=np.zeros((B, 3, H, W), np.float32))
    for hm in (np.full((B, 3, H, W), 0.25, np.float32),
               -np.random.default_rng(1).random((B, 3, H, W), dtype=np.float32)):
        got = runtime.decode(_t(hm, gpu), *(_t(maps[k], gpu) for k in ("off", "dir", "z", "dim")),
                             K=K).cpu().numpy()
        exp = decode_oracle.decode(hm, maps["off"], maps["dir"], maps["z"], maps["dim"], K=K)
        np.testing.assert_array_equal(got, exp)


def test_decode_without_offset(gpu):
    rng = np.random.default_rng(4)
    hm = rng.random((1, 3, 152, 152), dtype=np.float32)
    o = {k: rng.random(s, dtype=np.float32) for k, s in
         (("dir", (1, 2, 152, 152)), ("z", (1, 1, 152, 152)), ("dim", (1, 3, 152, 152)))}
    got = runtime.decode(_t(hm, gpu), None, _t(o["dir"], gpu), _t(o["z"], gpu), _t(o["dim"], gpu),
                         K=50).cpu().numpy()
    np.testing.assert_array_equal(got, decode_oracle.decode(hm, None, o["dir"], o["z"], o["dim"], K=50))


@pytest.mark.parametrize("B,C,H,W,K", [
    (3, 3, 37, 29, 50),      # odd bands (R = 5: 8 bands, last one 2 rows), halo rows at every cut
    (2, 3, 10, 10, 50),      # K > band pixels: per-band lists padded with sentinels
    (1, 1, 152, 152, 256),   # C * S * K limit: fewer bands
    (2, 16, 24, 24, 256),    # C * K = 4096: one band per class
    (1, 3, 3, 4100, 40),     # a band tile wider than LDS allows: the one-block-per-class kernels
    (2, 3, 152, 152, 50),    # production shape with quantised values: ties across band cuts
])
def test_decode_band_split_shapes(gpu, B, C, H, W, K):
    """The band-parallel decode (S row bands per class map, sorted band lists merged per frame)
    == the oracle's two topk stages bit for bit, on shapes that stress every band edge: odd
    heights, lists shorter than K, the C*S*K cap, the fallback kernels, plateaus and equal
    values crossing band cuts (quantised maps: many ties, ordered by lower index, then class)."""
    rng = np.random.default_rng(B * 1000 + H + W + K)
    hm = rng.random((B, C, H, W), dtype=np.float32)
    if (H, W) == (152, 152) and K == 50:
        hm = (np.floor(hm * 64) / 64).astype(np.float32)  # heavy ties, plateaus across cuts
        hm[:, :, 17:23, :] = np.float32(1.0)               # a 6-row plateau over the cut at row 19
    maps = {k: rng.standard_normal((B, c, H, W)).astype(np.float32)
            for k, c in (("off", 2), ("dir", 2), ("z", 1), ("dim", 3))}
    got = runtime.decode(_t(hm, gpu), *(_t(maps[k], gpu) for k in ("off", "dir", "z", "dim")),
                         K=K).cpu().numpy()
    exp = decode_oracle.decode(hm, maps["off"], maps["dir"], maps["z"], maps["dim"], K=K)
    np.testing.assert_array_equal(got, exp)
