"""KITTI constants of the hot path — every name and value of the reference's
config/kitti_config.py:7-87 (class ids, colours, front/back BEV boundaries, the BEV
raster, the voxel grid and the mean KITTI calibration with its inverses).
"""

import math

import numpy as np

from sfa_hip import dropin as _dropin

# class ids (config/kitti_config.py:7-17; the reference's duplicate 'Vehicle' key collapses)
CLASS_NAME_TO_ID = {
    "Pedestrian": 0, "Vehicle": 1, "Cyclist": 2, "Truck": -3, "Person_sitting": 0,
    "Tram": -99, "Misc": -99, "DontCare": -1,
}
colors = [[0, 255, 255], [0, 0, 255], [255, 0, 0], [255, 120, 0],
          [255, 120, 120], [0, 120, 0], [120, 255, 255], [120, 0, 255]]

# metric box of the front BEV crop (:23-30) and of the back crop (:36-43)
boundary = {"minX": 0, "maxX": 50, "minY": -25, "maxY": 25, "minZ": -2.73, "maxZ": 1.27}

bound_size_x = boundary["maxX"] - boundary["minX"]
bound_size_y = boundary["maxY"] - boundary["minY"]
bound_size_z = boundary["maxZ"] - boundary["minZ"]

boundary_back = {"minX": -50, "maxX": 0, "minY": -25, "maxY": 25, "minZ": -2.73, "maxZ": 1.27}

# BEV raster: rows along x, columns along y (:45-47)
BEV_WIDTH = 608
BEV_HEIGHT = 608
DISCRETIZATION = (boundary["maxX"] - boundary["minX"]) / BEV_HEIGHT

# max points per voxel (:50)
T = 35

# voxel size and grid (:53-60)
vd = 0.1
vh = 0.05
vw = 0.05
W = math.ceil(bound_size_x / vw)
H = math.ceil(bound_size_y / vh)
D = math.ceil(bound_size_z / vd)

# mean KITTI calibration (:64-83): velodyne -> reference camera, rectification, camera 2
Tr_velo_to_cam = np.array([
    [7.49916597e-03, -9.99971248e-01, -8.65110297e-04, -6.71807577e-03],
    [1.18652889e-02, 9.54520517e-04, -9.99910318e-01, -7.33152811e-02],
    [9.99882833e-01, 7.49141178e-03, 1.18719929e-02, -2.78557062e-01],
    [0, 0, 0, 1],
])
R0 = np.array([
    [0.99992475, 0.00975976, -0.00734152, 0],
    [-0.0097913, 0.99994262, -0.00430371, 0],
    [0.00729911, 0.0043753, 0.99996319, 0],
    [0, 0, 0, 1],
])
P2 = np.array([
    [719.787081, 0., 608.463003, 44.9538775],
    [0., 719.787081, 174.545111, 0.1066855],
    [0., 0., 1., 3.0106472e-03],
    [0., 0., 0., 0],
])

# inverses (:85-87), computed the same way (LAPACK inv / SVD pinv)
R0_inv = np.linalg.inv(R0)
Tr_velo_to_cam_inv = np.linalg.inv(Tr_velo_to_cam)
P2_inv = np.linalg.pinv(P2)


# names of the reference module this drop-in does not define come from the reference
__getattr__ = _dropin.module_getattr(__name__)
