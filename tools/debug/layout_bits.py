"""Are the bench's pipelines bit-identical in a given stream layout?  Builds bench.BevInferBench
with the given bench arguments (world 1), issues warm-up steps as the timed loop does, then one step
per pipeline, and compares each pipeline's head maps, intermediates (debug_views) and fp16x3 amax
words with pipeline 0 and with an eager forward of the same frames on a fresh engine.
    python tools/debug/layout_bits.py [bench args...]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from sfa_hip import _lib, runtime, synthetic  # noqa: E402

MAIN = os.environ.get("MAIN") == "1"
args = bench.parse(sys.argv[1:])
dev = torch.device("cuda", 0)
B, H, W = args.batch, 608, 608
if MAIN:  # bench.main() itself; the comparison runs in place of its --dump-dets step
    hooked = {}

    def hook(a, bb, rank, world):
        hooked["b"] = bb
        raise SystemExit(0)
    bench.dump_gathered = hook
    sys.argv = ["bench.py"] + sys.argv[1:] + ["--dump-dets", "/dev/null", "--probe-forwards", "0", "--no-cpu-baseline"]
    try:
        bench.main()
    except SystemExit:
        pass
    b = hooked["b"]
else:
    b = bench.BevInferBench(args, 0, 1, dev)
print("layout:", sys.argv[1:], "nf", b.nf, "side", b.side, "gather", b.gather)
for k in range(0 if MAIN else int(os.environ.get("WARM", 6))):
    b.one_step(k)
torch.cuda.synchronize()
if os.environ.get("TIMED"):  # bench main's timed loop: k restarts at 0, timing events per step
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(int(os.environ["TIMED"]))]
    for k in range(int(os.environ["TIMED"])):
        b.one_step(k, ev[k] if os.environ.get("EVENTS", "1") == "1" else None)
    torch.cuda.synchronize()


def amax_words(eng, ws):
    L = _lib.lib()
    off = int(L.sfa_forward_buffer_offset(eng._h, B, H, W, 9))  # heads L2
    nch = sum(c for _, c in eng.heads)
    off = (off + nch * B * (H // 4) * (W // 4) * 4 + 255) // 256 * 256
    w = ws[off: off + 21 * B * 256 * 4].view(torch.int32).cpu().numpy().reshape(21, B, 8, 32)
    return w.max(axis=2)  # the max over the shards (which shard a block commits to may vary)


def grab(p):
    v = p.engine.debug_views(p.ws, B, H, W)
    r = {}
    for k in ("layer1", "layer2", "layer3", "layer4", "up_level2", "up_level3", "up_level4"):
        r[k] = v[k].cpu().numpy()
    for j in range(3):
        for h in v["levels"]:
            r[f"L{j}/{h}"] = v["levels"][h][j].cpu().numpy()
    for h in p.outs:
        r["out/" + h] = p.outs[h].cpu().numpy()
    r["dets"] = p.dets.cpu().numpy()
    r["amax"] = amax_words(p.engine, p.ws)
    return r


res = []
for i in range(b.nf):
    b.one_step(i)
    torch.cuda.synchronize()
    res.append(grab(b.pipes[i]))
# eager reference on a fresh engine, one stream, no graph
arch = _lib.make_arch(runtime.DEFAULT_HEADS)
eng = runtime.KfpnEngine(arch, runtime.pack_state_dict(synthetic.synthetic_state_dict(_lib.state_layout(arch), 0), arch), dev)
eng.set_side_streams(False)
pipe = runtime.DetectorPipeline(eng, B, K=args.K)
pipe.x.copy_(b.pipes[0].x)
eng.forward_into(pipe.x, pipe.outs, _lib.IN_NCHW3, pipe.ws)
torch.cuda.synchronize()
ref = grab(pipe)
for i, r in enumerate(res):
    bad = [k for k in ref if k != "dets" and not np.array_equal(ref[k], r[k])]
    print(f"pipeline {i}: differs from eager in {len(bad)} tensors:", bad[:12])
    for k in bad[:4]:
        if k == "amax":
            w = np.argwhere(ref[k] != r[k])
            print("    amax slots/frames/words differing:", w[:12].tolist())
            for s, f, j in w[:6].tolist():
                print("      slot", s, "frame", f, "word", j, "eager", hex(int(ref[k][s, f, j]) & 0xffffffff), "pipe", hex(int(r[k][s, f, j]) & 0xffffffff))
        else:
            d = np.abs(ref[k].astype(np.float64) - r[k].astype(np.float64))
            fr = sorted(set(np.argwhere(d > 0)[:, 0].tolist()))
            print("   ", k, "max abs", float(np.nanmax(d)), "frames", fr[:16])
    print("   dets equal eager-pipeline decode? ", np.array_equal(r["dets"], res[0]["dets"]))
