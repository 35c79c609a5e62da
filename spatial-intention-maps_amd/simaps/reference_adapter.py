"""Read a reference VectorEnv (envs.py) into the scene format the device path consumes.

This is the glue a maintainer adds to the reference to switch VectorEnv.get_state() to the
device path.  It only READS attributes the reference objects already have:

  env.robots, env.robot_config, env.room_length / room_width, env.receptacle_position and the
      state-representation flags                                          envs.py:39-45, 59-61, 150-151
  robot.group_index, robot.get_position(), robot.get_heading(), robot.is_idle(),
      robot.waypoint_positions, robot.controller.waypoint_index,
      robot.target_end_effector_position, LiftingRobot.lift_state         envs.py:815-980, 1169-1282, 1475-1479
  robot.mapper.global_overhead_map_without_robots                         envs.py:2026
  robot.mapper.global_occupancy_map.occupancy_map                         envs.py:2029, 2417

No simulator or reference import is needed here; objects are duck-typed.
"""
import numpy as np

from . import constants as K

ROBOT_TYPE_BY_CLASS = {'LiftingRobot': 'lifting_robot', 'PushingRobot': 'pushing_robot',
                       'ThrowingRobot': 'throwing_robot', 'RescueRobot': 'rescue_robot'}


def robot_type(robot):
    for cls in type(robot).__mro__:
        if cls.__name__ in ROBOT_TYPE_BY_CLASS:
            return ROBOT_TYPE_BY_CLASS[cls.__name__]
    raise TypeError('not a reference robot class: %s' % type(robot).__name__)


_ROUNDING = []


def rotate_rounding():
    """How this process's numpy -- the one the reference's scipy.ndimage.rotate runs on -- rounds
    rotate's out_center ('fma' / 'plain', include/simaps.h SIMAPS_ROT_*); measured once."""
    if not _ROUNDING:
        _ROUNDING.append(K.host_rotate_rounding())
    return _ROUNDING[0]


def scene_from_env(env, with_maps=True):
    """The scene dict (simaps.synthetic format) of one reference VectorEnv at its current step."""
    flags = {k: getattr(env, k) for k in K.DEFAULT_FLAGS}
    H, W = K.padded_room_shape(env.room_width, env.room_length)
    robots = []
    for r in env.robots:
        typ = robot_type(r)
        # Robot.__init__ / Robot.reset leave these None until the robot's first action
        # (envs.py:828-832, 958-963; RobotController.__init__ 1373-1376): the reset state that
        # VectorEnv.reset() renders (envs.py:222), and every robot of a multi-robot env that has
        # not acted yet.  They are passed through as None (the robot is idle; batch.pack_descriptors
        # gives it no paths, and the render never reads them, as at envs.py:2305, 2363, 2371).
        wps, idx, tgt = r.waypoint_positions, r.controller.waypoint_index, r.target_end_effector_position
        robots.append({
            'type': typ, 'cls': K.ROBOT_TYPES.index(typ), 'group_index': int(r.group_index),
            'position': tuple(r.get_position()), 'heading': float(r.get_heading()),
            'lift_state': getattr(r, 'lift_state', None), 'idle': bool(r.is_idle()),
            'waypoint_positions': None if wps is None else [tuple(p) for p in wps],
            'waypoint_index': None if idx is None else int(idx),
            'target_ee': None if tgt is None else tuple(tgt),
        })
    scene = {
        'config': None, 'env_name': None, 'room_length': env.room_length, 'room_width': env.room_width,
        'flags': flags, 'robot_config': env.robot_config, 'H': H, 'W': W,
        'receptacle_position': getattr(env, 'receptacle_position', None), 'robots': robots,
        'rotate_rounding': rotate_rounding(),
    }
    if with_maps:
        scene['occupancy'] = np.stack([np.asarray(r.mapper.global_occupancy_map.occupancy_map, dtype=np.uint8)
                                       for r in env.robots])
        scene['overhead'] = np.stack([np.asarray(r.mapper.global_overhead_map_without_robots, dtype=np.float32)
                                      for r in env.robots])
    return scene


def awaiting_flags(env):
    """[robot.awaiting_new_action for robot in env.robots] (envs.py:322-323)."""
    return [bool(r.awaiting_new_action) for r in env.robots]
