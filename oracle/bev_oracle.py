"""BEV voxelisation oracle (numpy) — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates, with an independent algorithm (scatter-max instead of lexsort+unique):

* ``get_filtered_lidar``  — data_process/kitti_data_utils.py:228-251
  inclusive box test on every axis (:237-239), in float32 (numpy compares an f32
  array with a Python float in f32, NEP 50 and the pinned numpy 1.18 agree);
  then z <- z - minZ in float32 (:241).  Order preserved.
* ``makeBEVMap``          — data_process/kitti_bev_utils.py:22-55
  row  = int(floor(x_f32 / f32(D)))               (:28)
  col  = int(floor(y_f32 / f32(D)) + 304.5)       (:29, Width/2 with Width = 609)
  one "top" point per (row, col): max z; ties -> first in input order — what
  lexsort((-z, col, row)) + np.unique(return_index) selects (:32-35, both stable);
  height    = z_top / 4.0 in f32 stored to f64   (:43-44)
  intensity = i_top                               (:47)
  density   = min(1, ln(count+1)/ln(64)) in f64  (:46,48)
  (609, 609) maps cropped to [:608, :608] (:50-53): row/col 608 are dropped;
  negative rows (back boundary, never shifted by minX) wrap like numpy indexing.
  Channel order: [0]=intensity, [1]=height, [2]=density.
"""

from __future__ import annotations

import numpy as np

BEV_H = 608
BEV_W = 608
DISCRETIZATION = 50.0 / 608.0


def get_filtered_lidar(lidar: np.ndarray, boundary: dict) -> np.ndarray:
    f = np.float32
    x, y, z = lidar[:, 0], lidar[:, 1], lidar[:, 2]
    keep = ((x >= f(boundary["minX"])) & (x <= f(boundary["maxX"])) &
            (y >= f(boundary["minY"])) & (y <= f(boundary["maxY"])) &
            (z >= f(boundary["minZ"])) & (z <= f(boundary["maxZ"])))
    out = lidar[keep].astype(np.float32, copy=True)
    out[:, 2] = out[:, 2] - f(boundary["minZ"])
    return out


def cell_indices(pc: np.ndarray):
    """(row, col) int64 per point, before the 608-crop (kitti_bev_utils.py:28-29)."""
    d = np.float32(DISCRETIZATION)
    row = np.floor(pc[:, 0] / d).astype(np.int64)
    col = (np.floor(pc[:, 1] / d) + np.float32((BEV_W + 1) / 2)).astype(np.int64)
    return row, col


def makeBEVMap(pc: np.ndarray, boundary: dict) -> np.ndarray:
    n = pc.shape[0]
    out = np.zeros((3, BEV_H, BEV_W), dtype=np.float64)
    if n == 0:
        return out
    row, col = cell_indices(pc)
    row = np.where(row < 0, row + (BEV_H + 1), row)  # numpy negative-index wrap
    col = np.where(col < 0, col + (BEV_W + 1), col)
    z = pc[:, 2]
    cell = row * (BEV_W + 1) + col
    uniq, inv, counts = np.unique(cell, return_inverse=True, return_counts=True)
    zmax = np.full(uniq.size, -np.inf, dtype=np.float32)
    np.maximum.at(zmax, inv, z)
    first = np.full(uniq.size, n, dtype=np.int64)
    is_top = z == zmax[inv]
    np.minimum.at(first, inv[is_top], np.nonzero(is_top)[0])
    r = uniq // (BEV_W + 1)
    c = uniq % (BEV_W + 1)
    max_height = np.float32(float(np.abs(boundary["maxZ"] - boundary["minZ"])))
    height = (pc[first, 2] / max_height).astype(np.float32)
    inten = pc[first, 3]
    dens = np.minimum(1.0, np.log(counts + 1) / np.log(64))
    ok = (r < BEV_H) & (c < BEV_W)
    out[0, r[ok], c[ok]] = inten[ok]
    out[1, r[ok], c[ok]] = height[ok]
    out[2, r[ok], c[ok]] = dens[ok]
    return out


def density_lut_f32(n: int = 64) -> np.ndarray:
    """f32(min(1, ln(c+1)/ln 64)) for c = 0..n-1 (entry 0 unused: empty cell)."""
    c = np.arange(n, dtype=np.int64)
    lut = np.minimum(1.0, np.log(c + 1) / np.log(64))
    lut[0] = 0.0
    return lut.astype(np.float32)
