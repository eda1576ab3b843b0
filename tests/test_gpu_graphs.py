"""Captured HIP graphs of the forward stay bit-exact when other work runs between their replays
(round-6 finding).  With the models' side streams off — the N > 1, stream and fusion
layouts — a forward is a single-branch graph, and on this ROCm a captured hipMemsetAsync node (the
forward zeroed its fp16x3 amax words and split-K tickets with one) is replayed from a
kernel-argument slot that later launches reuse: replays after another engine's capture or an eager
forward zeroed some other address, left the tickets counting from garbage and put NaN into the FPN.
The forward now zeroes them with a kernel (aux_kernels.h launch_zero_words).  Each case: two
engines, their graphs, eager forwards interleaved; every replay equals the eager result bit for bit."""
import pytest
import torch

from sfa_hip import _lib, runtime, synthetic

pytestmark = pytest.mark.gpu

B = 16


def _setup(gpu):
    arch = _lib.make_arch(runtime.DEFAULT_HEADS)
    packed = runtime.pack_state_dict(synthetic.synthetic_state_dict(_lib.state_layout(arch), 0), arch)
    x = torch.from_numpy(synthetic.synthetic_bev(B, seed=1)).to(gpu)
    return arch, packed, x


def _pipe(arch, packed, x, gpu, side, opts=None):
    eng = runtime.KfpnEngine(arch, packed, gpu, side_streams=side)
    for k, v in (opts or {}).items():
        eng.set_option(k, v)
    p = runtime.DetectorPipeline(eng, B, K=50)
    p.x.copy_(x)
    return p


def _fwd(p):
    p.engine.forward_into(p.x, p.outs, _lib.IN_NCHW3, p.ws, _lib.stream_ptr(p.dev))


def _capture(p):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _fwd(p)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        _fwd(p)
    return g


def _snap(p):
    torch.cuda.synchronize()
    return {h: p.outs[h].clone() for h in p.outs}


def _equal(a, b):
    return all(torch.equal(a[h], b[h]) for h in a)


@pytest.mark.parametrize("side", [False, True])
@pytest.mark.parametrize("opts", [{}, {_lib.OPT_SPLITK_TICKETS: 0}])
def test_graph_replays_between_other_work(gpu, side, opts):
    arch, packed, x = _setup(gpu)
    a, b = _pipe(arch, packed, x, gpu, side, opts), _pipe(arch, packed, x, gpu, side, opts)
    _fwd(a)
    ref = _snap(a)
    ga = _capture(a)
    gb = _capture(b)  # another engine's eager warm-up + capture after ga
    seq = []
    for name, act, p in (("replay a", ga.replay, a), ("replay b", gb.replay, b), ("eager a", lambda: _fwd(a), a),
                         ("replay a after eager a", ga.replay, a), ("replay b after eager a", gb.replay, b),
                         ("eager b", lambda: _fwd(b), b), ("replay b after eager b", gb.replay, b),
                         ("replay a after eager b", ga.replay, a)):
        act()
        seq.append((name, _equal(_snap(p), ref)))
    assert all(ok for _, ok in seq), seq
