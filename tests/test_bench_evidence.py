"""bench.py reports PMC traffic only from a pass of the loaded library build:
the committed profiles/r*_pmc_forward_<math>.json whose lib_sha256 equals the library's sha256, else
null.  CPU only (no kernel runs)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def _pmc(tmp, name, sha, mb):
    d = {"lib_sha256": sha, "conv_hbm_bytes_per_forward": 123,
         "per_launch": [{"kernel": "sfa::conv_r3_kernel<256, 320, 32, 1, 1, 3, 1, 3766532>", "hbm_MB": mb}] * 3}
    with open(os.path.join(tmp, "profiles", name), "w") as f:
        json.dump(d, f)


def test_traffic_only_for_the_loaded_build(tmp_path, monkeypatch):
    os.makedirs(tmp_path / "profiles")
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    monkeypatch.setattr(bench, "_lib_sha256", lambda: "aaaa")
    args = bench.parse([])
    assert bench.head_traffic_per_launch(args) is None and bench.traffic_per_forward(args) is None
    _pmc(str(tmp_path), "r05z_pmc_forward_fp16x3.json", "bbbb", 100.0)  # another build
    assert bench.head_traffic_per_launch(args) is None and bench.traffic_per_forward(args) is None
    _pmc(str(tmp_path), "r06a_pmc_forward_fp16x3.json", "aaaa", 150.0)  # this build
    _pmc(str(tmp_path), "r06b_pmc_forward_fp16x3.json", "cccc", 200.0)  # newer, another build
    ht = bench.head_traffic_per_launch(args)
    assert ht["bytes"] == 150_000_000 and ht["file"].endswith("r06a_pmc_forward_fp16x3.json")
    assert bench.traffic_per_forward(args) == 123
    line = bench.roofline_line(args, [0.4, 0.6, 0.3], {"achieved": 1.0}, 1.0, 833.0, "x", 628.0)
    assert line["traffic"] == 150_000_000 and "sha256 matched" in line["traffic_basis"]
    monkeypatch.setattr(bench, "_lib_sha256", lambda: "dddd")
    line = bench.roofline_line(args, [0.4, 0.6, 0.3], {"achieved": 1.0}, 1.0, 833.0, "x", 628.0)
    assert line["traffic"] is None and line["traffic_basis"].startswith("null")


def test_committed_pmc_pass_matches_the_shipped_library():
    """The newest committed forward PMC pass describes the library in the tree (rebuilds are
    reproducible: the same sources give the same sha256)."""
    import glob
    if not os.path.isfile(bench._lib.LIB_PATH):
        import pytest
        pytest.skip("library not built")
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_forward_fp16x3.json")))
    shas = [json.load(open(f)).get("lib_sha256") for f in files]
    assert bench._lib_sha256() in shas, "re-run tools/pmc_forward.sh on this build and commit its summary"
