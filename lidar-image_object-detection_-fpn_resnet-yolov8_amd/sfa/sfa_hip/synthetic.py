"""Deterministic synthetic inputs: weights, BEV tensors and LiDAR clouds.

Nothing here depends on a checkpoint or a dataset (neither ships offline,
SURVEY.md §8(c)).  Every value is a pure function of (seed, stream, counter)
through a splitmix64 counter hash, so the golden-fixture generator, the GPU
tests and ``bench.py`` all rebuild bit-identical inputs without files.

* ``synthetic_state_dict`` — the SURVEY §8(c)(i) weight conditioning:
  conv weights He-uniform ±sqrt(6/fan_in), conv biases U(-0.1, 0.1),
  BN gamma U(0.5, 1), beta U(-0.1, 0.1), running_mean U(-0.1, 0.1),
  running_var U(0.5, 2).  This spreads the top-K heatmap scores far enough
  apart (≈60 ulp) that index parity is well defined; PyTorch's default init
  produces ties (SURVEY §7 hard part 2).
* ``synthetic_point_cloud`` — the SURVEY §8(d) cloud: 64 rings x 1,920
  azimuths plus 20 boxes x 500 points = 132,880 points, float32 xyzi.
* ``synthetic_bev`` — U[0,1) BEV batch (conv throughput is value independent).
"""

from __future__ import annotations

import zlib

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def hash_uniform(seed: int, stream: int, n: int) -> np.ndarray:
    """n float64 values in [0, 1) from counter hash (seed, stream, i)."""
    with np.errstate(over="ignore"):
        key = _splitmix64(np.array([(seed * 0x100000001B3 + stream) & 0xFFFFFFFFFFFFFFFF],
                                   dtype=np.uint64))[0]
        ctr = np.arange(n, dtype=np.uint64) + key
        bits = _splitmix64(ctr)
    return (bits >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def hash_normal(seed: int, stream: int, n: int) -> np.ndarray:
    """n standard normals (Box-Muller over two hash streams)."""
    u1 = hash_uniform(seed, stream * 2 + 1, n)
    u2 = hash_uniform(seed, stream * 2 + 2, n)
    return np.sqrt(-2.0 * np.log1p(-u1)) * np.cos(2.0 * np.pi * u2)


def _name_stream(name: str) -> int:
    return zlib.crc32(name.encode("utf-8"))


def synthetic_tensor(name: str, shape, seed: int = 0) -> np.ndarray:
    """Value of one state_dict entry under the SURVEY §8(c)(i) conditioning."""
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    u = hash_uniform(seed, _name_stream(name), n)
    leaf = name.rsplit(".", 1)[-1]
    # BatchNorm entries are recognised by their buffer names / parent module.
    is_bn = (".bn" in name or name.startswith("bn") or ".downsample.1." in name)
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    if leaf == "running_mean":
        v = -0.1 + 0.2 * u
    elif leaf == "running_var":
        v = 0.5 + 1.5 * u
    elif leaf == "weight" and is_bn:
        v = 0.5 + 0.5 * u
    elif leaf == "bias" and is_bn:
        v = -0.1 + 0.2 * u
    elif leaf == "weight":  # conv weight (O, I, kh, kw)
        fan_in = int(np.prod(shape[1:]))
        a = np.sqrt(6.0 / fan_in)
        v = -a + 2.0 * a * u
    elif leaf == "bias":  # conv bias
        v = -0.1 + 0.2 * u
    else:
        raise KeyError(f"unknown state entry {name}")
    return v.reshape(shape).astype(np.float32)


def synthetic_state_dict(spec, seed: int = 0) -> dict:
    """spec: iterable of (name, shape) -> {name: np.ndarray}."""
    return {name: synthetic_tensor(name, shape, seed) for name, shape in spec}


def synthetic_bev(batch: int, height: int = 608, width: int = 608, seed: int = 1) -> np.ndarray:
    """(B, 3, H, W) float32 in [0, 1) — the bench's synthetic BEV batch."""
    return hash_uniform(seed, 7, batch * 3 * height * width).astype(np.float32).reshape(
        batch, 3, height, width)


def synthetic_logits(shape, seed: int, stream: int, scale: float = 3.0) -> np.ndarray:
    """Gaussian logits used as decode inputs (continuous -> tie-free)."""
    n = int(np.prod(shape))
    return (scale * hash_normal(seed, stream, n)).astype(np.float32).reshape(shape)


def synthetic_point_cloud(seed: int = 1, n_elev: int = 64, n_azim: int = 1920,
                          n_boxes: int = 20, pts_per_box: int = 500) -> np.ndarray:
    """SURVEY §8(d) synthetic KITTI-like sweep: (N, 4) float32 x, y, z, intensity."""
    el = np.deg2rad(np.linspace(-24.8, 2.0, n_elev))
    az = np.linspace(-np.pi, np.pi, n_azim, endpoint=False)
    EL, AZ = np.meshgrid(el, az, indexing="ij")
    EL = EL.ravel()
    AZ = AZ.ravel()
    n_ring = EL.size
    with np.errstate(divide="ignore"):
        r = np.where(EL < 0, np.minimum(1.73 / np.tan(-np.minimum(EL, -1e-12)), 80.0), 80.0)
    r = r + 0.05 * hash_normal(seed, 101, n_ring)
    x = r * np.cos(EL) * np.cos(AZ)
    y = r * np.cos(EL) * np.sin(AZ)
    z = r * np.sin(EL)
    inten = hash_uniform(seed, 102, n_ring)
    ring = np.stack([x, y, z, inten], axis=1)

    nb = n_boxes * pts_per_box
    cx = 5.0 + 40.0 * hash_uniform(seed, 103, n_boxes)
    cy = -20.0 + 40.0 * hash_uniform(seed, 104, n_boxes)
    bid = np.repeat(np.arange(n_boxes), pts_per_box)
    bx = cx[bid] + (-2.0 + 4.0 * hash_uniform(seed, 105, nb))
    by = cy[bid] + (-1.0 + 2.0 * hash_uniform(seed, 106, nb))
    bz = -1.73 + 1.73 * hash_uniform(seed, 107, nb)
    bi = hash_uniform(seed, 108, nb)
    boxes = np.stack([bx, by, bz, bi], axis=1)
    return np.concatenate([ring, boxes], axis=0).astype(np.float32)
