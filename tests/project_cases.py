"""Seeded inputs for the post-processing / camera-projection fixtures,
shared by tests/golden/gen_project_golden.py and the tests.

dets are (B, K, 10) f32 in sfa_decode's column order [score, xs, ys, z, dim0, dim1, dim2,
dir0, dir1, cls] with realistic magnitudes (xs/ys on the 152x152 head grid, metres for
z/dims), so the projected boxes land in, across and outside the image.  Calibrations are
float32 matrices, as Calibration.read_calib_file returns them (kitti_data_utils.py:149-165).
"""

import numpy as np

from sfa_hip import synthetic

# kitti_config.py:62-84 averages, as a calib file would hold them (f32)
_TR = np.array([[7.49916597e-03, -9.99971248e-01, -8.65110297e-04, -6.71807577e-03],
                [1.18652889e-02, 9.54520517e-04, -9.99910318e-01, -7.33152811e-02],
                [9.99882833e-01, 7.49141178e-03, 1.18719929e-02, -2.78557062e-01]])
_R0 = np.array([[0.99992475, 0.00975976, -0.00734152],
                [-0.0097913, 0.99994262, -0.00430371],
                [0.00729911, 0.0043753, 0.99996319]])
_P2 = np.array([[719.787081, 0., 608.463003, 44.9538775],
                [0., 719.787081, 174.545111, 0.1066855],
                [0., 0., 1., 3.0106472e-03]])
# a second, typical KITTI raw-sequence calibration
_P2B = np.array([[721.5377, 0., 609.5593, 44.85728],
                 [0., 721.5377, 172.854, 0.2163791],
                 [0., 0., 1., 0.002745884]])
_TRB = np.array([[7.533745e-03, -9.999714e-01, -6.166020e-04, -4.069766e-03],
                 [1.480249e-02, 7.280733e-04, -9.998902e-01, -7.631618e-02],
                 [9.998621e-01, 7.523790e-03, 1.480755e-02, -2.717806e-01]])
_R0B = np.array([[9.999239e-01, 9.837760e-03, -7.445048e-03],
                 [-9.869795e-03, 9.999421e-01, -4.278459e-03],
                 [7.402527e-03, 4.351614e-03, 9.999631e-01]])


def calibs():
    """name -> dict(V2C, R0, P2 as f32 arrays, img_shape (rows, cols))."""
    f = lambda a: np.asarray(a, np.float32)
    return {"avg": dict(V2C=f(_TR), R0=f(_R0), P2=f(_P2), img_shape=(375, 1242)),
            "seq": dict(V2C=f(_TRB), R0=f(_R0B), P2=f(_P2B), img_shape=(370, 1224))}


def _dets(seed, B, K):
    u = lambda s, n: synthetic.hash_uniform(seed, s, n).reshape(B, K)
    d = np.zeros((B, K, 10), np.float32)
    d[..., 0] = u(1, B * K)                       # score
    d[..., 1] = u(2, B * K) * 152                 # xs (BEV column -> lidar y)
    d[..., 2] = u(3, B * K) * 152                 # ys (BEV row -> lidar x, forward)
    d[..., 3] = 0.8 + u(4, B * K) * 1.6           # z (+ minZ -> about -1.9 .. -0.3 m)
    d[..., 4] = 1.2 + u(5, B * K) * 1.0           # h
    d[..., 5] = 0.5 + u(6, B * K) * 2.0           # w (m)
    d[..., 6] = 0.6 + u(7, B * K) * 4.4           # l (m)
    d[..., 7] = u(8, B * K) * 2 - 1               # dir im
    d[..., 8] = u(9, B * K) * 2 - 1               # dir re
    d[..., 9] = np.floor(u(10, B * K) * 3)        # class 0..2
    return d


def cases():
    c = {"typical": (_dets(31, 4, 50), ["avg", "seq", "avg", "seq"])}
    e = _dets(32, 3, 40)
    e[0, :, 9] = 0                                # class 0 only: all dropped by the 0.3 quirk
    e[1, :8, 0] = np.float32(0.2)                 # exactly peak_thresh: dropped (strict >)
    e[1, 8:16, 0] = np.nextafter(np.float32(0.2), np.float32(1))
    e[1, 16:24, 2] = np.linspace(0, 3, 8)          # within a few metres of the sensor
    e[1, 24:32, 1] = np.array([0, 1, 2, 150, 151, 152, 75, 76], np.float32)  # lateral edges
    e[1, 32:40, 7:9] = np.array([[0, 1], [1, 0], [0, -1], [-1, 0], [0, 0], [1, 1], [-1, -1],
                                 [1e-8, -1]], np.float32)  # yaw quadrants, atan2(0, 0)
    e[2, :, 0] = np.float32(0.1)                  # nothing passes peak_thresh
    c["edges"] = (e, ["seq", "avg", "avg"])
    return c
