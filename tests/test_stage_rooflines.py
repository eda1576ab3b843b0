"""tools/stage_rooflines.py: the per-launch FLOP plan adds up to bench.py's algorithmic work, and the
committed table of the shipped library is regenerated from the committed evidence unchanged."""
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import stage_rooflines  # noqa: E402


def test_plan_flop_matches_bench_constant():
    import bench
    plan = stage_rooflines.forward_plan()
    assert len(plan) == 32  # the launches of one fp16x3 forward at 608^2 (rocprof issue order)
    flop = 0.0
    for pair in (1, 2, 3):  # an FPN pair is charged one reference conv, split over its two launches
        flops = {f for (_, _, f, p) in plan if p == pair}
        assert len(flops) == 1
        flop += flops.pop()
    flop += sum(f for (_, _, f, p) in plan if f and p is None)
    # heads: the bench line's per-level FLOP (3x3 conv + the 1x1 heads), as bench.head_flop_per_launch
    s4, s8 = 16 * 152 * 152, 16 * 76 * 76
    heads = sum(2.0 * m * 320 * 9 * c + 2.0 * m * 11 * 64 for m, c in ((s8, 256), (s4, 128), (s4, 64)))
    assert abs(flop + heads - bench.CONV_FLOP_PER_FRAME * 16) / (bench.CONV_FLOP_PER_FRAME * 16) < 1e-9


def test_committed_table_regenerates(tmp_path):
    tables = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_stage_rooflines.txt")))
    assert tables
    newest = tables[-1]
    tag = os.path.basename(newest).split("_")[0]
    prof = os.path.join(REPO, "profiles", f"{tag}_prof_summary_probe_serial.txt")
    pmc = os.path.join(REPO, "profiles", f"{tag}_pmc_forward_fp16x3.json")
    bj = os.path.join(REPO, "profiles", f"{tag}_bench_probe_serial.json")
    out = tmp_path / "t.txt"
    old = os.getcwd()
    os.chdir(REPO)
    try:
        stage_rooflines.main([os.path.relpath(prof), os.path.relpath(pmc), os.path.relpath(bj), "--out", str(out)])
    finally:
        os.chdir(old)
    assert out.read_text() == open(newest).read()
