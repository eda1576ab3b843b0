"""KITTI BEV geometry used by the hot path (mirror of the reference's
config/kitti_config.py:7-47, constants only — same names and values).
"""

import math  # noqa: F401

# class ids (config/kitti_config.py:7-17)
CLASS_NAME_TO_ID = {
    "Pedestrian": 0, "Vehicle": 1, "Cyclist": 2, "Truck": -3, "Person_sitting": 0,
    "Tram": -99, "Misc": -99, "DontCare": -1,
}
colors = [[0, 255, 255], [0, 0, 255], [255, 0, 0], [255, 120, 0],
          [255, 120, 120], [0, 120, 0], [120, 255, 255], [120, 0, 255]]

# metric box of the front BEV crop (:23-30) and of the back crop (:36-43)
boundary = dict(minX=0, maxX=50, minY=-25, maxY=25, minZ=-2.73, maxZ=1.27)
boundary_back = dict(minX=-50, maxX=0, minY=-25, maxY=25, minZ=-2.73, maxZ=1.27)

bound_size_x = boundary["maxX"] - boundary["minX"]
bound_size_y = boundary["maxY"] - boundary["minY"]
bound_size_z = boundary["maxZ"] - boundary["minZ"]

# BEV raster: rows along x, columns along y (:45-47)
BEV_WIDTH = 608
BEV_HEIGHT = 608
DISCRETIZATION = (boundary["maxX"] - boundary["minX"]) / BEV_HEIGHT

# max points per voxel (:50)
T = 35
