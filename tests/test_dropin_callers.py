"""The drop-in boundary for the reference's callers (north_star: "test.py and demo_front.py
are drop-in").

The reference's scripts append their own ``sfa`` dir to sys.path and then import
(``test.py:20-28``, ``demo_front.py:30-37``, ``demo_2_sides.py:27-34``) a mix of hot-path
names and names this build does not provide.  With the drop-in root FIRST on sys.path,
every one of those import statements must succeed, the hot-path names must come from the
drop-in and the others from the reference's own files (``sfa_hip/dropin.py``), and
``config.kitti_config`` must equal the reference's name for name, value for value.

The import statements are read from the callers with ``ast`` (parsed, not executed) and
performed one by one with importlib in a fresh interpreter, with stub ``cv2`` / ``easydict``
/ ``wget`` modules (absent here; the callers need them only for drawing, configs and the
demo download).  The reference is copied to a scratch dir named ``sfa`` (its modules walk
up to a directory named ``sfa``).  Build container only: skipped where
``/root/reference`` is absent (the GPU box).
"""

from __future__ import annotations

import ast
import json
import os
import shutil
import subprocess
import sys
import textwrap

import pytest

from conftest import SFA_ROOT

REF = "/root/reference"
CALLERS = ("test.py", "demo_front.py", "demo_2_sides.py")
PKGS = ("models", "utils", "config", "data_process")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "data_process")),
                                reason="reference tree not present (GPU box)")

# names the drop-in itself must serve (the hot path and its host API)
DROPIN_NAMES = {
    ("models.model_utils", "create_model"),
    ("utils.evaluation_utils", "decode"),
    ("utils.evaluation_utils", "post_processing"),
    ("utils.evaluation_utils", "draw_predictions"),
    ("utils.evaluation_utils", "convert_det_to_real_values"),
    ("utils.torch_utils", "_sigmoid"),
    ("data_process.kitti_data_utils", "Calibration"),
    ("utils.demo_utils", "do_detect"),
    ("utils.demo_utils", "parse_demo_configs"),
    ("utils.demo_utils", "download_and_unzip"),
    ("utils.demo_utils", "write_credit"),
}

_STUBS = {
    "cv2.py": """
        FONT_HERSHEY_SIMPLEX = 0
        LINE_AA = 16
        def _nop(*a, **k):
            return None
        putText = polylines = line = imshow = imwrite = resize = rectangle = _nop
        def waitKey(*a, **k):
            return 27
    """,
    "easydict.py": """
        class EasyDict(dict):
            def __getattr__(self, k):
                try:
                    return self[k]
                except KeyError:
                    raise AttributeError(k)
            def __setattr__(self, k, v):
                self[k] = v
    """,
    "wget.py": """
        def download(url, out=None):
            raise RuntimeError("no network")
    """,
}

_RUNNER = r"""
import importlib, json, os, sys
import numpy as np
dropin_root, stubs, ref_root, imports = sys.argv[1], sys.argv[2], sys.argv[3], json.loads(sys.argv[4])
sys.path[:0] = [dropin_root, stubs]            # INTEGRATION.md: drop-in root first
sys.path.append(ref_root)                       # what the caller's src_dir walk appends
res = {"resolved": [], "errors": []}
for mod, names in imports:
    try:
        m = importlib.import_module(mod)
    except Exception as e:
        res["errors"].append(f"import {mod}: {type(e).__name__}: {e}")
        continue
    for n in names:
        try:
            obj = getattr(m, n)
        except Exception as e:
            res["errors"].append(f"from {mod} import {n}: {type(e).__name__}: {e}")
            continue
        src = getattr(sys.modules.get(getattr(obj, "__module__", "") or "", None), "__file__", None)
        res["resolved"].append([mod, n, os.path.realpath(src) if src else None,
                                os.path.realpath(m.__file__)])
# config.kitti_config against the reference's own module
import importlib.util
spec = importlib.util.spec_from_file_location("_ref_cnf", os.path.join(ref_root, "config", "kitti_config.py"))
ref = importlib.util.module_from_spec(spec); spec.loader.exec_module(ref)
import config.kitti_config as cnf
cmp = {}
for k, v in vars(ref).items():
    if k.startswith("__") or type(v).__name__ == "module":
        continue
    if not hasattr(cnf, k):
        cmp[k] = "missing"; continue
    w = getattr(cnf, k)
    if isinstance(v, np.ndarray):
        ok = isinstance(w, np.ndarray) and w.dtype == v.dtype and w.shape == v.shape and np.array_equal(w, v)
    else:
        ok = type(w) is type(v) and w == v
    cmp[k] = "ok" if ok else f"differs: {w!r} vs {v!r}"
res["kitti_config"] = cmp
print("@@" + json.dumps(res))
"""


def _caller_imports(path):
    """Module-level imports after the caller's ``sys.path.append(src_dir)`` block, of the
    reference's packages: [(module, [names])] (``import a.b as c`` -> (a.b, []))."""
    tree = ast.parse(open(path).read(), filename=path)
    out = []
    for node in tree.body:
        if isinstance(node, ast.ImportFrom) and node.module and node.module.split(".")[0] in PKGS:
            out.append((node.module, [a.name for a in node.names]))
        elif isinstance(node, ast.ImportFrom) and node.module in PKGS:
            out.append((node.module, [a.name for a in node.names]))
        elif isinstance(node, ast.Import):
            for a in node.names:
                if a.name.split(".")[0] in PKGS:
                    out.append((a.name, []))
    return out


@pytest.fixture(scope="module")
def ref_tree(tmp_path_factory):
    base = tmp_path_factory.mktemp("dropin")
    root = base / "ref" / "sfa"
    for d in PKGS:
        shutil.copytree(os.path.join(REF, d), root / d, ignore=shutil.ignore_patterns("__pycache__"))
    stubs = base / "stubs"
    stubs.mkdir()
    for name, body in _STUBS.items():
        (stubs / name).write_text(textwrap.dedent(body))
    return str(root), str(stubs)


@pytest.mark.parametrize("caller", CALLERS)
def test_caller_import_block_resolves(caller, ref_tree):
    ref_root, stubs = ref_tree
    imports = _caller_imports(os.path.join(REF, caller))
    assert len(imports) >= 7, imports
    env = dict(os.environ)
    env.pop("SFA_REFERENCE_ROOT", None)
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    r = subprocess.run([sys.executable, "-c", _RUNNER, SFA_ROOT, stubs, ref_root, json.dumps(imports)],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(os.path.dirname(ref_root)))
    line = [x for x in r.stdout.splitlines() if x.startswith("@@")]
    assert r.returncode == 0 and line, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(line[0][2:])
    assert res["errors"] == [], res["errors"]
    dropin = os.path.realpath(SFA_ROOT)
    n_dropin = n_ref = 0
    for mod, name, src, modfile in res["resolved"]:
        # every package the caller names is the drop-in's
        if (mod, name) in DROPIN_NAMES:
            assert src and src.startswith(dropin), (mod, name, src)
            n_dropin += 1
        elif mod in ("config.kitti_config",) or name == "":
            continue
        else:
            # out-of-scope names resolve to the reference's own files
            assert src is None or src.startswith(ref_root) or src.startswith(dropin), (mod, name, src)
            if src and src.startswith(ref_root):
                n_ref += 1
    assert n_dropin >= 2 and n_ref >= 2, res["resolved"]
    bad = {k: v for k, v in res["kitti_config"].items() if v != "ok"}
    assert bad == {}, bad


def test_fallthrough_names_and_hot_path_owner(ref_tree):
    """Specific resolutions: hot-path modules are the drop-in's files; the modules this build
    does not provide are the reference's; a name missing from a shadowed module comes from
    the reference's module of the same name (kitti_dataset.py:17 imports gen_hm_radius)."""
    ref_root, stubs = ref_tree
    probe = r"""
import importlib, json, os, sys
sys.path[:0] = [sys.argv[1], sys.argv[2]]; sys.path.append(sys.argv[3])
out = {}
for m in ["models.model_utils", "models.fpn_resnet", "utils.evaluation_utils", "utils.torch_utils",
          "data_process.kitti_bev_utils", "data_process.kitti_data_utils", "config.kitti_config",
          "utils.demo_utils", "data_process.kitti_dataloader", "data_process.kitti_dataset",
          "data_process.transformation", "data_process.demo_dataset", "utils.misc", "utils.visualization_utils"]:
    out[m] = os.path.realpath(importlib.import_module(m).__file__)
import data_process.kitti_data_utils as kdu
out["gen_hm_radius"] = kdu.gen_hm_radius.__module__
import data_process.kitti_dataset as kds
out["kitti_dataset.makeBEVMap"] = kds.makeBEVMap.__module__
try:
    kdu.no_such_name
    out["missing"] = "resolved?!"
except AttributeError as e:
    out["missing"] = "AttributeError"
print("@@" + json.dumps(out))
"""
    r = subprocess.run([sys.executable, "-c", probe, SFA_ROOT, stubs, ref_root], capture_output=True,
                       text=True, timeout=300)
    line = [x for x in r.stdout.splitlines() if x.startswith("@@")]
    assert r.returncode == 0 and line, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(line[0][2:])
    dropin = os.path.realpath(SFA_ROOT)
    for m in ["models.model_utils", "models.fpn_resnet", "utils.evaluation_utils", "utils.torch_utils",
              "data_process.kitti_bev_utils", "data_process.kitti_data_utils", "config.kitti_config",
              "utils.demo_utils", "data_process.kitti_dataloader", "data_process.kitti_dataset"]:
        assert out[m].startswith(dropin), (m, out[m])
    for m in ["data_process.transformation", "data_process.demo_dataset", "utils.misc", "utils.visualization_utils"]:
        assert out[m].startswith(ref_root), (m, out[m])
    assert out["gen_hm_radius"] == "_sfa_reference.data_process.kitti_data_utils"
    # names the drop-in dataset module does not define come from the reference's module, whose
    # own imports bind the drop-in's (HIP) voxeliser
    assert out["kitti_dataset.makeBEVMap"] == "data_process.kitti_bev_utils"
    assert out["missing"] == "AttributeError"


def test_calibration_parses_like_reference(tmp_path, ref_tree):
    """Calibration (kitti_data_utils.py:94-173) on a KITTI-format calib file: same arrays,
    dtypes and intrinsics as the reference's class."""
    ref_root, stubs = ref_tree
    rows = ["P0: " + " ".join(["1.0"] * 12), "P1: " + " ".join(["2.0"] * 12),
            "P2: 7.215377e+02 0.000000e+00 6.095593e+02 4.485728e+01 0.000000e+00 7.215377e+02 "
            "1.728540e+02 2.163791e-01 0.000000e+00 0.000000e+00 1.000000e+00 2.745884e-03",
            "P3: " + " ".join(f"{0.5 * i:.6e}" for i in range(12)),
            "R0_rect: 9.999239e-01 9.837760e-03 -7.445048e-03 -9.869795e-03 9.999421e-01 "
            "-4.278459e-03 7.402527e-03 4.351614e-03 9.999631e-01",
            "Tr_velo_to_cam: 7.533745e-03 -9.999714e-01 -6.166020e-04 -4.069766e-03 1.480249e-02 "
            "7.280733e-04 -9.998902e-01 -7.631618e-02 9.998621e-01 7.523790e-03 1.480755e-02 -2.717806e-01",
            "Tr_imu_to_velo: " + " ".join(["0.0"] * 12)]
    calib = tmp_path / "calib.txt"
    calib.write_text("\n".join(rows) + "\n")
    probe = r"""
import importlib.util, json, os, sys
import numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]; sys.path.append(sys.argv[3])
from data_process.kitti_data_utils import Calibration
spec = importlib.util.spec_from_file_location("_ref_kdu", os.path.join(sys.argv[3], "data_process", "kitti_data_utils.py"))
ref = importlib.util.module_from_spec(spec); spec.loader.exec_module(ref)
a, b = Calibration(sys.argv[4]), ref.Calibration(sys.argv[4])
bad = []
for k in ("P2", "P3", "V2C", "R0", "c_u", "c_v", "f_u", "f_v", "b_x", "b_y"):
    x, y = np.asarray(getattr(a, k)), np.asarray(getattr(b, k))
    if x.dtype != y.dtype or x.shape != y.shape or not np.array_equal(x, y):
        bad.append(k)
p = np.arange(12, dtype=np.float32).reshape(4, 3)
if not np.array_equal(a.cart2hom(p), b.cart2hom(p)) or a.cart2hom(p).dtype != b.cart2hom(p).dtype:
    bad.append("cart2hom")
print("@@" + json.dumps(bad))
"""
    r = subprocess.run([sys.executable, "-c", probe, SFA_ROOT, stubs, ref_root, str(calib)],
                       capture_output=True, text=True, timeout=300)
    line = [x for x in r.stdout.splitlines() if x.startswith("@@")]
    assert r.returncode == 0 and line, r.stdout[-3000:] + r.stderr[-3000:]
    assert json.loads(line[0][2:]) == []


def test_parse_demo_configs_matches_reference(ref_tree, tmp_path):
    """parse_demo_configs (demo_utils.py:36-93): identical configuration dict."""
    ref_root, stubs = ref_tree
    probe = r"""
import importlib.util, json, os, sys
sys.path[:0] = [sys.argv[1], sys.argv[2]]; sys.path.append(sys.argv[3])
sys.argv = ["demo", "--K", "40", "--gpu_idx", "1"]
from utils.demo_utils import parse_demo_configs
mine = dict(parse_demo_configs())
spec = importlib.util.spec_from_file_location("_ref_du", os.path.join(sys.path[-1], "utils", "demo_utils.py"))
ref = importlib.util.module_from_spec(spec); spec.loader.exec_module(ref)
theirs = dict(ref.parse_demo_configs())
print("@@" + json.dumps({"mine": {k: repr(v) for k, v in mine.items()},
                          "theirs": {k: repr(v) for k, v in theirs.items()}}))
"""
    r = subprocess.run([sys.executable, "-c", probe, SFA_ROOT, stubs, ref_root], capture_output=True,
                       text=True, timeout=300, cwd=str(tmp_path))
    line = [x for x in r.stdout.splitlines() if x.startswith("@@")]
    assert r.returncode == 0 and line, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(line[0][2:])
    assert out["mine"] == out["theirs"]


def test_reference_root_without_sfa_ancestor_is_skipped(tmp_path):
    """A reference tree not under a '*sfa' dir would hang the reference's own src_dir walk:
    the fall-through skips it (with a warning) instead of importing from it."""
    fake = tmp_path / "plain"
    (fake / "models").mkdir(parents=True)
    (fake / "data_process").mkdir()
    (fake / "models" / "fpn_resnet.py").write_text("")
    (fake / "data_process" / "kitti_bev_utils.py").write_text("")
    probe = r"""
import json, sys, warnings
sys.path.insert(0, sys.argv[1])
from sfa_hip import dropin
import os
os.environ["SFA_REFERENCE_ROOT"] = sys.argv[2]
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    roots = dropin.reference_roots()
print("@@" + json.dumps({"roots": list(roots), "warned": len(w)}))
"""
    r = subprocess.run([sys.executable, "-c", probe, SFA_ROOT, str(fake)], capture_output=True,
                       text=True, timeout=300)
    line = [x for x in r.stdout.splitlines() if x.startswith("@@")]
    assert r.returncode == 0 and line, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(line[0][2:])
    assert out["roots"] == [] and out["warned"] == 1
