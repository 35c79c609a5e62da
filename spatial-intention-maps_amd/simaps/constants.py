"""Geometry / encoding constants of the observation path, restated from the reference.

Every value is the reference's own constant (file:line relative to the reference repo root);
nothing here is tuned.  Pure Python, no numpy/torch import, so both the python3.9 golden
generator and the product host code can use it.
"""
import math

# Mapper (envs.py:2010-2013)
LOCAL_MAP_PIXEL_WIDTH = 96
LOCAL_MAP_WIDTH = 1
LOCAL_MAP_PIXELS_PER_METER = LOCAL_MAP_PIXEL_WIDTH / LOCAL_MAP_WIDTH  # 96.0 (a float, as in the reference)

# VectorEnv (envs.py:23-27)
WALL_HEIGHT = 0.1
CUBE_WIDTH = 0.044
RECEPTACLE_WIDTH = 0.15

# Robot (envs.py:802-810) and subclasses (PushingRobot 1059-1062, ThrowingRobot 1279-1282,
# LiftingRobot 1169-1171; Rescue/Lifting use RobotWithHooks -> Robot geometry).
HALF_WIDTH = 0.03
BACKPACK_OFFSET = -0.0135
BASE_LENGTH = 0.065
END_EFFECTOR_LOCATION = BACKPACK_OFFSET + BASE_LENGTH
RADIUS = math.sqrt(HALF_WIDTH ** 2 + END_EFFECTOR_LOCATION ** 2)
LIFTED_CUBE_OFFSET = -0.007

ROBOT_TYPES = ('lifting_robot', 'pushing_robot', 'throwing_robot', 'rescue_robot')
CLS_LIFTING, CLS_PUSHING, CLS_THROWING, CLS_RESCUE = range(4)


def _geom(base_length):
    ee = BACKPACK_OFFSET + base_length
    return {'BASE_LENGTH': base_length, 'END_EFFECTOR_LOCATION': ee,
            'RADIUS': math.sqrt(HALF_WIDTH ** 2 + ee ** 2)}


ROBOT_GEOM = {
    'lifting_robot': _geom(BASE_LENGTH),
    'pushing_robot': _geom(BASE_LENGTH + 0.005),   # envs.py:1060 (5 mm blade)
    'throwing_robot': _geom(BASE_LENGTH + 0.006),  # envs.py:1280 (6 mm offset)
    'rescue_robot': _geom(BASE_LENGTH),
}

# Camera.SEG_VALUES (envs.py:1881-1890)
SEG_VALUES = {
    'floor': 1.0 / 8, 'obstacle': 2.0 / 8, 'receptacle': 3.0 / 8, 'cube': 4.0 / 8,
    'robot_group_1': 5.0 / 8, 'robot_group_2': 6.0 / 8, 'robot_group_3': 7.0 / 8, 'robot_group_4': 8.0 / 8,
}

# VectorEnv.__init__ defaults for the state-representation flags (envs.py:39-45)
# OccupancyMap.selem_thin = disk(ceil(Robot.HALF_WIDTH * 96)) (envs.py:2426), HALF_WIDTH = 0.03 (envs.py:802)
THIN_RADIUS_PX = 3

DEFAULT_FLAGS = {
    'use_robot_map': True,
    'use_distance_to_receptacle_map': False,
    'distance_to_receptacle_map_scale': 0.25,
    'use_shortest_path_to_receptacle_map': True,
    'use_shortest_path_map': True,
    'shortest_path_map_scale': 0.25,
    'use_intention_map': False,
    'intention_map_encoding': 'ramp',
    'intention_map_scale': 1.0,
    'intention_map_line_thickness': 2,
    'use_history_map': False,
    'use_intention_channels': False,
    'intention_channel_encoding': 'spatial',
    'intention_channel_nonspatial_scale': 0.025,
}

INTENTION_ENCODINGS = ('ramp', 'binary', 'line', 'circle')


def round_up_to_even(x):
    """Mapper.round_up_to_even (envs.py:2405-2407)."""
    return 2 * math.ceil(x / 2)


def padded_room_shape(room_width, room_length):
    """Mapper.create_padded_room_zeros shape (envs.py:2383-2389)."""
    return (round_up_to_even(room_width * LOCAL_MAP_PIXELS_PER_METER + math.sqrt(2) * LOCAL_MAP_PIXEL_WIDTH),
            round_up_to_even(room_length * LOCAL_MAP_PIXELS_PER_METER + math.sqrt(2) * LOCAL_MAP_PIXEL_WIDTH))


def room_rect(room_width, room_length):
    """OccupancyMap._create_room_mask rectangle (envs.py:2468-2476) -> (i0, j0, h, w)."""
    H, W = padded_room_shape(room_width, room_length)
    room_length_pixels = round_up_to_even((room_length - 2 * HALF_WIDTH) * LOCAL_MAP_PIXELS_PER_METER)
    room_width_pixels = round_up_to_even((room_width - 2 * HALF_WIDTH) * LOCAL_MAP_PIXELS_PER_METER)
    start_i = int(H / 2 - room_width_pixels / 2)
    start_j = int(W / 2 - room_length_pixels / 2)
    return start_i, start_j, room_width_pixels, room_length_pixels


def cspace_radius_px(robot_type):
    """OccupancyMap selem radius: disk(floor(RADIUS * 96)) (envs.py:2421)."""
    return math.floor(ROBOT_GEOM[robot_type]['RADIUS'] * LOCAL_MAP_PIXELS_PER_METER)


def crop_width():
    """Mapper._get_local_map crop width round_up_to_even(sqrt(2)*96) = 136 (envs.py:2202)."""
    return round_up_to_even(math.sqrt(2) * LOCAL_MAP_PIXEL_WIDTH)


def room_dims(env_name):
    """utils.apply_misc_env_modifications (utils.py:166-175): (room_length, room_width, num_cubes)."""
    if env_name.startswith('large'):
        return 1.0, 1.0, 20
    return 1.0, 0.5, 10


# scipy.ndimage.rotate (envs.py:2206, 2267) computes out_center = rot_matrix @ ((S - 1) / 2) with
# numpy matmul -> BLAS dgemv (scipy/ndimage/interpolation.py:928 in scipy 1.7.1).  Whether that
# dgemv fuses M[r][0] * a0 into the second product's sum (an FMA kernel) is a property of the
# numpy / OpenBLAS build and the host CPU, and it decides the sample grid of ~4 % of headings.
ROTATE_ROUNDINGS = ('fma', 'plain')


_HOST_ROUNDING = []


def scene_rotate_rounding(scene):
    """The rotate rounding a scene renders with: its own 'rotate_rounding' entry (synthetic scenes,
    the reference adapter and the golden fixtures record it), else this process's numpy rounding --
    what the reference's scipy.ndimage.rotate would use here (measured once per process)."""
    r = scene.get('rotate_rounding')
    if r is not None:
        return r
    if not _HOST_ROUNDING:
        _HOST_ROUNDING.append(host_rotate_rounding())
    return _HOST_ROUNDING[0]


def host_rotate_rounding():
    """'fma' or 'plain': how THIS process's numpy rounds rot_matrix @ v, i.e. what
    scipy.ndimage.rotate does on this host.  Measured on rotation matrices / half-integer
    vectors of the same shape as rotate's, with exact rational arithmetic for the two candidate
    forms; raises if the host follows neither."""
    from fractions import Fraction
    import numpy as np
    rs = np.random.RandomState(2206)
    votes = {'fma': 0, 'plain': 0}
    n = 0
    for t in rs.uniform(-math.pi, math.pi, 256):
        c, s = math.cos(t), math.sin(t)
        a = np.array([float(rs.randint(60, 200)) / 2, float(rs.randint(60, 200)) / 2])
        got = np.array([[c, s], [-s, c]]) @ a
        for r, (m0, m1) in enumerate(((c, s), (-s, c))):
            n += 1
            votes['fma'] += float(got[r]) == float(Fraction(m0) * Fraction(a[0]) + Fraction(m1 * a[1]))
            votes['plain'] += float(got[r]) == m0 * a[0] + m1 * a[1]
    for k in ROTATE_ROUNDINGS:
        if votes[k] == n:
            return k
    raise RuntimeError('numpy matmul rounds rot_matrix @ v in neither the fused nor the plain form '
                       '(%d / %d / %d): the drop-in cannot reproduce this host\'s scipy.ndimage.rotate' % (
                           votes['fma'], votes['plain'], n))


def position_to_pixel_indices(x, y, shape):
    """Mapper.position_to_pixel_indices (envs.py:2391-2397) of one position given as Python floats
    (float64 arithmetic, as numpy does for them): (i, j) ints, clipped to the grid."""
    i = math.floor(shape[0] / 2 - y * LOCAL_MAP_PIXELS_PER_METER)
    j = math.floor(shape[1] / 2 + x * LOCAL_MAP_PIXELS_PER_METER)
    return min(max(i, 0), shape[0] - 1), min(max(j, 0), shape[1] - 1)
