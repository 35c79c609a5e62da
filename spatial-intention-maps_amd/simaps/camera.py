"""Camera model of the observation ingest, host side.

Robot.update_map -> Mapper.update (envs.py:2056-2066): the robot's camera image (pybullet depth
buffer + segmentation mask) becomes a point cloud (Camera.capture_image, envs.py:1927-1955),
which is scattered into the robot's overhead map (highest point per pixel wins: argsort by z,
last write) and, for obstacle points, into its occupancy map (OccupancyMap.update, 2447-2450).

This module holds the per-camera constants and the per-robot camera pose (_get_camera_params,
envs.py:1974-2008), evaluated with Python's math exactly like the reference; everything per point
runs on the GPU (simaps_ingest).
"""
import math

import numpy as np

from . import constants as K

ROBOT_HEIGHT = 0.07          # Robot.HEIGHT (envs.py:809)
ROBOT_BACKPACK_OFFSET = -0.0135
ROBOT_TOP_LENGTH = 0.057     # envs.py:803-806
FOV = 60                     # Camera.FOV, vertical (envs.py:1880)


class CameraSpec:
    def __init__(self, name, aspect, near, far):
        self.name, self.aspect, self.near, self.far = name, aspect, near, far
        self.height_px = int(1.63 * K.LOCAL_MAP_PIXEL_WIDTH)    # envs.py:1895
        self.width_px = int(self.aspect * self.height_px)       # envs.py:1896
        limit_y = math.tan(math.radians(FOV / 2))               # envs.py:1944
        limit_x = limit_y * self.aspect
        self.cx2, self.cy2 = 2 * limit_x, 2 * limit_y           # pixel_x / pixel_y scales (envs.py:1946-1947)

    def params(self, x, y, heading):
        """_get_camera_params(robot_position, robot_heading) -> 9 floats (position, target, up)."""
        if self.name == 'overhead':  # OverheadCamera (envs.py:1974-1978)
            pos = (x, y, 1)
            tgt = (x, y, 0)
            up = (math.cos(heading), math.sin(heading), 0)
        else:  # ForwardFacingCamera (envs.py:1990-2008)
            off = ROBOT_BACKPACK_OFFSET + ROBOT_TOP_LENGTH + 0.002
            pos = (x + off * math.cos(heading), y + off * math.sin(heading), ROBOT_HEIGHT)
            toff = ROBOT_HEIGHT * math.tan(math.radians(90 + -30))
            tgt = (pos[0] + toff * math.cos(heading), pos[1] + toff * math.sin(heading), 0)
            up = (math.cos(math.radians(90 + -30)) * math.cos(heading),
                  math.cos(math.radians(90 + -30)) * math.sin(heading),
                  math.sin(math.radians(90 + -30)))
        return [float(v) for v in pos + tgt + up]

    def params_batch(self, poses):
        """params() of every (x, y, heading) in `poses` as an [n, 9] float64 array, bitwise equal:
        cos / sin come from Python's math per robot (numpy's SIMD kernels may round differently),
        the rest is the same IEEE products and sums, elementwise."""
        p = np.asarray(poses, dtype=np.float64).reshape(-1, 3)
        x, y = p[:, 0], p[:, 1]
        ch = np.array([math.cos(h) for h in p[:, 2].tolist()], dtype=np.float64)
        sh = np.array([math.sin(h) for h in p[:, 2].tolist()], dtype=np.float64)
        out = np.empty((len(p), 9), dtype=np.float64)
        if self.name == 'overhead':
            out[:, 0], out[:, 1], out[:, 2] = x, y, 1.0
            out[:, 3], out[:, 4], out[:, 5] = x, y, 0.0
            out[:, 6], out[:, 7], out[:, 8] = ch, sh, 0.0
        else:
            off = ROBOT_BACKPACK_OFFSET + ROBOT_TOP_LENGTH + 0.002
            toff = ROBOT_HEIGHT * math.tan(math.radians(90 + -30))
            cu = math.cos(math.radians(90 + -30))
            out[:, 0] = x + off * ch
            out[:, 1] = y + off * sh
            out[:, 2] = ROBOT_HEIGHT
            out[:, 3] = out[:, 0] + toff * ch
            out[:, 4] = out[:, 1] + toff * sh
            out[:, 5] = 0.0
            out[:, 6], out[:, 7] = cu * ch, cu * sh
            out[:, 8] = math.sin(math.radians(90 + -30))
        return out


# ForwardFacingCamera (use_partial_observations, envs.py:2019-2022, 1980-1985) / OverheadCamera (1965-1969)
FORWARD = CameraSpec('forward', 16.0 / 9, 0.001, 1)
OVERHEAD = CameraSpec('overhead', 1, 0.1, 10)
CAMERAS = {'forward': FORWARD, 'overhead': OVERHEAD}
