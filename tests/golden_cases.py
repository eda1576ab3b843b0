"""Shared regeneration of golden-fixture INPUTS (outputs come from the .npz files).

Mirrors tests/golden/gen_golden.py's case definitions without needing the reference.
"""
import numpy as np

from sfa_hip import synthetic

BOUNDARY = {"minX": 0, "maxX": 50, "minY": -25, "maxY": 25, "minZ": -2.73, "maxZ": 1.27}
HEADS = {"hm_cen": 3, "cen_offset": 2, "direction": 2, "z_coor": 1, "dim": 3}
DECODE_CASES = {"b2_152_k50": (2, 152, 152, 50, 11), "b3_64_k40": (3, 64, 64, 40, 12),
                "b1_32_k20_plateau": (1, 32, 32, 20, 13)}
MODEL_CASES = {"b2_96": (2, 96, 96, 21), "b1_160x128": (1, 160, 128, 22)}


def bev_cases(golden_bev):
    """(name, cloud) — sweeps are regenerated from seeds, KAT clouds read from the fixture."""
    out = [("sweep_s1", synthetic.synthetic_point_cloud(1)),
           ("sweep_s2_sub", synthetic.synthetic_point_cloud(2)[::7].copy())]
    for name in ("kat_edges", "single_point", "empty_after_filter"):
        out.append((name, golden_bev[f"{name}/cloud"]))
    return out


def decode_inputs(case):
    B, H, W, K, seed = DECODE_CASES[case]
    hm = synthetic.synthetic_logits((B, 3, H, W), seed, 1, 1.0 if "plateau" not in case else 3.0)
    if "plateau" in case:
        hm = np.round(hm * 2.0) / 2.0
    off = synthetic.synthetic_logits((B, 2, H, W), seed, 2)
    dirn = synthetic.synthetic_logits((B, 2, H, W), seed, 3, 1.0)
    z = synthetic.synthetic_logits((B, 1, H, W), seed, 4, 1.0)
    dim = synthetic.synthetic_logits((B, 3, H, W), seed, 5, 1.0)
    return dict(hm=hm, off=off, dir=dirn, z=z, dim=dim, K=K)


def model_input(case):
    B, H, W, seed = MODEL_CASES[case]
    return synthetic.hash_uniform(seed, 7, B * 3 * H * W).astype(np.float32).reshape(B, 3, H, W)


def state_spec(golden_model):
    names = [str(n) for n in golden_model["state_names"]]
    shapes = [tuple(int(v) for v in s if v > 0) for s in golden_model["state_shapes"]]
    return [(n, () if n.endswith("num_batches_tracked") else s) for n, s in zip(names, shapes)]


def state_dict_np(golden_model, seed=0):
    return synthetic.synthetic_state_dict(state_spec(golden_model), seed)
