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


# ---- the reference's decode helpers on their own (evaluation_utils.py:21-74): the drop-in serves
# them from sfa_heat_nms / sfa_topk / sfa_gather_feat, checked against the oracle's restatements

def _scores(B, C, H, W, seed, ties=False):
    rng = np.random.default_rng(seed)
    s = rng.permutation(B * C * H * W).astype(np.float32).reshape(B, C, H, W) / (B * C * H * W)  # tie-free
    if ties:
        s = np.round(s * 64) / 64  # heavy ties: the order is the documented (index, class) one
    return s.astype(np.float32)


@pytest.mark.parametrize("shape", [(2, 3, 152, 152), (1, 3, 37, 53), (2, 1, 7, 9)])
def test_nms_helper_bit_exact(gpu, shape):
    from utils.evaluation_utils import _nms
    h = _scores(*shape, seed=3, ties=True)  # plateaus: every member of a plateau survives
    got = _nms(_t(h, gpu))
    assert got.shape == h.shape and got.device == gpu
    np.testing.assert_array_equal(got.cpu().numpy(), decode_oracle.nms_peaks(h))


@pytest.mark.parametrize("shape,K", [((2, 3, 152, 152), 50), ((3, 3, 64, 64), 40), ((2, 16, 100, 100), 200),
                                     ((1, 2, 5, 5), 25)])
@pytest.mark.parametrize("ties", [False, True])
def test_topk_helpers_match_oracle(gpu, shape, K, ties):
    """_topk / _topk_channel: the band kernels (152 x 152, 64 x 64) and the one-block-per-class
    fallback (16 classes x K = 200 over 100 x 100: no band split fits), K = H*W included; with ties the
    order is lower flat index, then lower class (torch leaves it unspecified)."""
    from utils.evaluation_utils import _topk, _topk_channel
    s = _scores(*shape, seed=sum(shape) + K, ties=ties)
    sc, ind, cls, ys, xs = (t.cpu().numpy() for t in _topk(_t(s, gpu), K=K))
    esc, eind, ecls, eys, exs = decode_oracle.topk(s, K)
    np.testing.assert_array_equal(sc, esc)
    np.testing.assert_array_equal(ind, eind)
    np.testing.assert_array_equal(cls, ecls)
    np.testing.assert_array_equal(ys, eys)
    np.testing.assert_array_equal(xs, exs)
    assert ind.dtype == np.int64 and cls.dtype == np.int32 and ys.dtype == np.float32
    B, C, H, W = shape
    csc, cind, cys, cxs = (t.cpu().numpy() for t in _topk_channel(_t(s, gpu), K=K))
    assert csc.shape == (B, C, K)
    flat = s.reshape(B, C, H * W)
    for b in range(B):
        for c in range(C):
            v, i = decode_oracle._topk_desc(flat[b, c], K)
            np.testing.assert_array_equal(csc[b, c], v)
            np.testing.assert_array_equal(cind[b, c], i)
            np.testing.assert_array_equal(cys[b, c], (i // W).astype(np.float32))
            np.testing.assert_array_equal(cxs[b, c], (i % W).astype(np.float32))
    with pytest.raises(RuntimeError):
        _topk(_t(s, gpu), K=H * W + 1)


def test_gather_helpers_bit_exact(gpu):
    from utils.evaluation_utils import _gather_feat, _transpose_and_gather_feat
    rng = np.random.default_rng(8)
    feat = rng.standard_normal((3, 4, 21, 19)).astype(np.float32)
    ind = rng.integers(0, 21 * 19, (3, 37)).astype(np.int64)
    got = _transpose_and_gather_feat(_t(feat, gpu), _t(ind, gpu)).cpu().numpy()
    np.testing.assert_array_equal(got, decode_oracle._gather(feat, ind))
    flat = rng.standard_normal((3, 50, 6)).astype(np.float32)
    ind2 = rng.integers(0, 50, (3, 11)).astype(np.int64)
    exp = np.stack([flat[b][ind2[b]] for b in range(3)])
    np.testing.assert_array_equal(_gather_feat(_t(flat, gpu), _t(ind2, gpu)).cpu().numpy(), exp)
    # int64 features (the _topk stage-2 gathers of topk_inds), bit for bit
    big = rng.integers(-2 ** 62, 2 ** 62, (2, 30, 1)).astype(np.int64)
    ind3 = rng.integers(0, 30, (2, 9)).astype(np.int64)
    np.testing.assert_array_equal(_gather_feat(_t(big, gpu), _t(ind3, gpu)).cpu().numpy(),
                                  np.stack([big[b][ind3[b]] for b in range(2)]))
    with pytest.raises(RuntimeError):
        _gather_feat(_t(flat, gpu), _t(np.full((3, 2), 50, np.int64), gpu))
    with pytest.raises(NotImplementedError):
        _gather_feat(_t(flat, gpu), _t(ind2, gpu), mask=torch.ones((3, 11), dtype=torch.bool, device=gpu))


def test_sigmoid_non_contiguous_in_place(gpu):
    """_sigmoid on a strided view (the reference's in-place sigmoid_ accepts any tensor): the view's
    elements are updated in place, the rest of the storage is untouched, the same object returned."""
    from utils.torch_utils import _sigmoid
    rng = np.random.default_rng(4)
    base = rng.standard_normal((2, 6, 33, 35)).astype(np.float32)
    t = _t(base, gpu)
    view = t[:, 1:5].transpose(2, 3)
    assert not view.is_contiguous()
    out = _sigmoid(view)
    assert out is view
    exp = base.copy()
    exp[:, 1:5] = decode_oracle.sigmoid_clamp(base[:, 1:5])
    got = t.cpu().numpy()
    np.testing.assert_array_equal(got[:, [0, 5]], base[:, [0, 5]])
    assert float(np.max(np.abs(got - exp))) <= 2 * np.finfo(np.float32).eps
