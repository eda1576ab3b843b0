"""GPU parity of BEV voxelisation + point filter vs the reference fixtures (bit-exact)."""
import hashlib

import numpy as np
import pytest
import torch

import golden_cases as gc
from oracle import bev_oracle
from sfa_hip import _lib, runtime

pytestmark = pytest.mark.gpu

NAMES = ["sweep_s1", "sweep_s2_sub", "kat_edges", "single_point", "empty_after_filter"]


def _scratch_clean(vox):
    """The voxeliser's scratch contract: zero again after every call, except the binned path's
    record region (written before it is read, never assumed zero). Layout (csrc/bev.hip):
    atomic keys + counts per cell, then the binned counters [count | offset | cursor], then the
    records."""
    B = vox.max_batch
    al = lambda n: (n + 255) // 256 * 256  # noqa: E731
    atomic = al(B * 608 * 608 * 8) + al(B * 608 * 608 * 4)
    bins = 3 * al(B * 76 * 4)
    return int(vox.scratch[:atomic + bins].count_nonzero()) == 0


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", NAMES)
def test_make_bev_map_f64_bit_exact(golden, gpu, name):
    from data_process.kitti_bev_utils import makeBEVMap
    from data_process.kitti_data_utils import get_filtered_lidar
    g = golden.bev
    cloud = dict(gc.bev_cases(g))[name]
    filt = get_filtered_lidar(cloud, gc.BOUNDARY)  # HIP compaction
    assert filt.shape[0] == int(g[f"{name}/filtered_n"])
    assert _sha(filt) == str(g[f"{name}/filtered_sha"])
    bev = makeBEVMap(filt, gc.BOUNDARY)  # HIP voxeliser, f64 like the reference
    assert bev.dtype == np.float64 and bev.shape == (3, 608, 608)
    assert _sha(bev) == str(g[f"{name}/map_sha"])


def test_raw_batch_layouts_bit_exact(golden, gpu):
    """Fused filter+voxelise on a ragged batch, all three output layouts."""
    g = golden.bev
    clouds = [c for _, c in gc.bev_cases(g)]
    offs = np.cumsum([0] + [c.shape[0] for c in clouds])
    pts = torch.from_numpy(np.concatenate(clouds)).to(gpu)
    vox = runtime.BevVoxelizer(gpu, len(clouds))
    f64 = vox(pts, offs, gc.BOUNDARY, layout=_lib.BEV_NCHW3_F64).cpu().numpy()
    f32 = vox(pts, offs, gc.BOUNDARY, layout=_lib.BEV_NCHW3_F32).cpu().numpy()
    nhwc = vox(pts, offs, gc.BOUNDARY, layout=_lib.BEV_NHWC4_F32).cpu().numpy()
    for b, name in enumerate(NAMES):
        assert _sha(f64[b]) == str(g[f"{name}/map_sha"]), name
        np.testing.assert_array_equal(f32[b], f64[b].astype(np.float32))
        np.testing.assert_array_equal(nhwc[b][..., :3].transpose(2, 0, 1), f32[b])
        assert np.all(nhwc[b][..., 3] == 0)


def test_scratch_stays_clean_and_repeatable(gpu):
    from sfa_hip import synthetic
    clouds = [synthetic.synthetic_point_cloud(s) for s in (3, 4)]
    offs = np.cumsum([0] + [c.shape[0] for c in clouds])
    pts = torch.from_numpy(np.concatenate(clouds)).to(gpu)
    vox = runtime.BevVoxelizer(gpu, 2)
    a = vox(pts, offs, gc.BOUNDARY, layout=_lib.BEV_NCHW3_F64).cpu().numpy()
    assert _scratch_clean(vox)
    b = vox(pts, offs, gc.BOUNDARY, layout=_lib.BEV_NCHW3_F64).cpu().numpy()
    np.testing.assert_array_equal(a, b)
    for i, c in enumerate(clouds):
        exp = bev_oracle.makeBEVMap(bev_oracle.get_filtered_lidar(c, gc.BOUNDARY), gc.BOUNDARY)
        np.testing.assert_array_equal(a[i], exp)


def test_shuffled_ties_follow_input_order(gpu):
    """Equal max-z points in a cell: the FIRST in input order supplies intensity."""
    rng = np.random.default_rng(5)
    n = 20000
    pts = np.zeros((n, 4), np.float32)
    pts[:, 0] = rng.uniform(10, 10.3, n)
    pts[:, 1] = rng.uniform(-0.3, 0.3, n)
    pts[:, 2] = rng.choice(np.float32([-1.0, 0.5]), n)
    pts[:, 3] = rng.uniform(0, 1, n)
    exp = bev_oracle.makeBEVMap(bev_oracle.get_filtered_lidar(pts, gc.BOUNDARY), gc.BOUNDARY)
    got = runtime.BevVoxelizer(gpu, 1)(torch.from_numpy(pts).to(gpu), [0, n], gc.BOUNDARY,
                                       layout=_lib.BEV_NCHW3_F64).cpu().numpy()[0]
    np.testing.assert_array_equal(got, exp)


def test_back_boundary_wraps_like_numpy(gpu):
    """boundary_back: rows never shifted by minX -> negative numpy indices wrap."""
    from sfa_hip import synthetic
    back = {"minX": -50, "maxX": 0, "minY": -25, "maxY": 25, "minZ": -2.73, "maxZ": 1.27}
    c = synthetic.synthetic_point_cloud(6)
    filt = bev_oracle.get_filtered_lidar(c, back)
    exp = bev_oracle.makeBEVMap(filt, back)
    got = runtime.BevVoxelizer(gpu, 1)(torch.from_numpy(c).to(gpu), [0, c.shape[0]], back,
                                       layout=_lib.BEV_NCHW3_F64).cpu().numpy()[0]
    np.testing.assert_array_equal(got, exp)


def test_filter_large_random(gpu):
    rng = np.random.default_rng(9)
    n = 1_000_003
    pts = rng.uniform(-60, 60, (n, 4)).astype(np.float32)
    pts[:, 2] = rng.uniform(-4, 3, n)
    got = runtime.filter_points(torch.from_numpy(pts).to(gpu), gc.BOUNDARY).cpu().numpy()
    np.testing.assert_array_equal(got, bev_oracle.get_filtered_lidar(pts, gc.BOUNDARY))


def test_cpu_input_refused():
    with pytest.raises(_lib.SfaNativeError):
        runtime.filter_points(torch.zeros(4, 4), gc.BOUNDARY)


@pytest.mark.parametrize("flip", [False, True])
def test_binned_path_equals_atomic_path(gpu, flip):
    """The default blocked voxeliser (one pass bins each 1024 points by 4-row strips into its own
    record region + table, each strip reduced in LDS), the same with 8-row strips
    (SFA_BEV_STRIP8) and round 2's binned one (count / scan /
    bin / strip, SFA_BEV_FORCE_BINNED) give the bits of the global-atomic one (flag SFA_BEV_FORCE_ATOMIC) in every layout, flipped or not,
    on a ragged batch with a saturated-density cell and an empty frame; both leave the scratch
    zeroed."""
    from sfa_hip import synthetic
    rng = np.random.default_rng(11)
    dense = np.zeros((5000, 4), np.float32)  # one cell, > 63 points (density cap), z ties
    dense[:, 0] = 20.01
    dense[:, 1] = 0.01
    dense[:, 2] = rng.choice(np.float32([-1.5, 0.25, 0.25]), 5000)
    dense[:, 3] = rng.uniform(0, 1, 5000)
    clouds = [synthetic.synthetic_point_cloud(s) for s in (7, 8)] + [dense, np.zeros((0, 4), np.float32),
                                                                      synthetic.synthetic_point_cloud(9)]
    offs = np.cumsum([0] + [c.shape[0] for c in clouds])
    pts = torch.from_numpy(np.concatenate(clouds)).to(gpu)
    vox = runtime.BevVoxelizer(gpu, len(clouds))
    flags = _lib.BEV_RAW | (_lib.BEV_FLIP_HW if flip else 0)
    for layout in (_lib.BEV_NCHW3_F64, _lib.BEV_NCHW3_F32, _lib.BEV_NHWC4_F32):
        blocked = vox(pts, offs, gc.BOUNDARY, layout=layout, flags=flags).cpu().numpy()
        assert _scratch_clean(vox)
        strip8 = vox(pts, offs, gc.BOUNDARY, layout=layout, flags=flags | _lib.BEV_STRIP8).cpu().numpy()
        assert _scratch_clean(vox)
        binned = vox(pts, offs, gc.BOUNDARY, layout=layout, flags=flags | _lib.BEV_FORCE_BINNED).cpu().numpy()
        assert _scratch_clean(vox)
        atomic = vox(pts, offs, gc.BOUNDARY, layout=layout, flags=flags | _lib.BEV_FORCE_ATOMIC).cpu().numpy()
        assert _scratch_clean(vox)
        np.testing.assert_array_equal(blocked, atomic)
        np.testing.assert_array_equal(strip8, atomic)
        np.testing.assert_array_equal(binned, atomic)
    f64 = vox(pts, offs, gc.BOUNDARY, layout=_lib.BEV_NCHW3_F64).cpu().numpy()
    for i, c in enumerate(clouds):
        exp = bev_oracle.makeBEVMap(bev_oracle.get_filtered_lidar(c, gc.BOUNDARY), gc.BOUNDARY)
        np.testing.assert_array_equal(f64[i], exp)


def test_oversized_frame_uses_atomic_path(gpu):
    """A batch with more points than the scratch holds as records (here 1 frame of 400,000 points,
    capacity ~277 k) takes the global-atomic path: still bit-exact, scratch still clean."""
    rng = np.random.default_rng(13)
    n = 400_000
    pts = np.zeros((n, 4), np.float32)
    pts[:, 0] = rng.uniform(-1, 51, n)
    pts[:, 1] = rng.uniform(-26, 26, n)
    pts[:, 2] = rng.uniform(-3, 1.5, n)
    pts[:, 3] = rng.uniform(0, 1, n)
    vox = runtime.BevVoxelizer(gpu, 1)
    assert n * 16 > vox.scratch.numel() // 2  # the record region: the half after the atomic cells
    got = vox(torch.from_numpy(pts).to(gpu), [0, n], gc.BOUNDARY, layout=_lib.BEV_NCHW3_F64).cpu().numpy()[0]
    assert _scratch_clean(vox)
    exp = bev_oracle.makeBEVMap(bev_oracle.get_filtered_lidar(pts, gc.BOUNDARY), gc.BOUNDARY)
    np.testing.assert_array_equal(got, exp)


def test_scratch_shared_across_batch_sizes(gpu):
    """One scratch (sized for 8 frames, as runtime.voxelizer() shares it) serves calls of every
    batch size and path in any order: the layout follows the scratch's capacity, not the call's
    batch, so a small call's records never land in a later larger call's zero areas (ADVICE r03:
    B = 1 blocked, then B = 4 atomic / B = 2 binned / a frame over 1 M points)."""
    from sfa_hip import synthetic
    rng = np.random.default_rng(17)
    huge = np.zeros((1_200_000, 4), np.float32)  # > 1024 regions of one frame: not the blocked path
    huge[:, 0] = rng.uniform(-1, 51, huge.shape[0])
    huge[:, 1] = rng.uniform(-26, 26, huge.shape[0])
    huge[:, 2] = rng.uniform(-3, 1.5, huge.shape[0])
    huge[:, 3] = rng.uniform(0, 1, huge.shape[0])
    sweeps = [synthetic.synthetic_point_cloud(s) for s in range(20, 28)]
    exp = {}

    def oracle(c):
        k = id(c)
        if k not in exp:
            exp[k] = bev_oracle.makeBEVMap(bev_oracle.get_filtered_lidar(c, gc.BOUNDARY), gc.BOUNDARY)
        return exp[k]

    vox = runtime.BevVoxelizer(gpu, 8)
    calls = [(sweeps[:1], 0), (sweeps[1:5], _lib.BEV_FORCE_ATOMIC), (sweeps[:1], 0),
             (sweeps[2:4], _lib.BEV_FORCE_BINNED), (sweeps[:1], _lib.BEV_STRIP8), (sweeps, 0),
             (sweeps[:1], 0), ([sweeps[5], huge, sweeps[6]], 0), (sweeps[:2], 0),
             ([huge], _lib.BEV_FORCE_ATOMIC), (sweeps[3:8], 0)]
    for clouds, flags in calls:
        offs = np.cumsum([0] + [c.shape[0] for c in clouds])
        pts = torch.from_numpy(np.concatenate(clouds)).to(gpu)
        got = vox(pts, offs, gc.BOUNDARY, layout=_lib.BEV_NCHW3_F64, flags=flags).cpu().numpy()
        assert _scratch_clean(vox), (len(clouds), flags)
        for i, c in enumerate(clouds):
            np.testing.assert_array_equal(got[i], oracle(c), err_msg=f"B={len(clouds)} flags={flags} frame {i}")
