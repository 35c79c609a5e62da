"""Seeded synthetic scenes for the observation path.

There is no PyBullet here: a scene is what the observation path reads from the simulator
at one step -- per-robot poses / controller state, and per-agent observed global maps
(occupancy u8 and overhead-without-robots f32).  Geometry follows the reference:
walls / divider / room corners (envs.py:515-649), receptacle (envs.py:150-151, 469-477),
cubes (envs.py:26, 686-692), robot spawn (envs.py:651-716), intention/history paths
(RobotController.get_intention_path / get_history_path, envs.py:1475-1479).

Pure numpy (no torch): imported by the python3.9 golden generator, by the tests and by bench.py.
"""
import math

import numpy as np

from . import constants as K

# The five BASELINE.json configs (+ flag variants from config/experiments/comparisons/**,
# used only as extra parity cases).  Flags are the reference's YAML values.
_BASE_FLAGS = dict(K.DEFAULT_FLAGS)

CONFIGS = {
    # config/experiments/base/lifting_1-small_empty-base.yml
    'lifting_1-small_empty': dict(env_name='small_empty', robot_config=[{'lifting_robot': 1}], flags={}),
    # config/experiments/ours/lifting_4-small_divider-ours.yml
    'lifting_4-small_divider': dict(env_name='small_divider', robot_config=[{'lifting_robot': 4}],
                                    flags={'use_intention_map': True}),
    # config/experiments/ours/pushing_4-large_empty-ours.yml
    'pushing_4-large_empty': dict(env_name='large_empty', robot_config=[{'pushing_robot': 4}],
                                  flags={'use_intention_map': True}),
    # config/experiments/ours/lifting_2_throwing_2-large_empty-ours.yml
    'lifting_2_throwing_2-large_empty': dict(env_name='large_empty',
                                             robot_config=[{'lifting_robot': 2}, {'throwing_robot': 2}],
                                             flags={'use_intention_map': True}),
    # config/experiments/ours/rescue_4-small_empty-ours.yml (utils.py:177-180 drops receptacle maps)
    'rescue_4-small_empty': dict(env_name='small_empty', robot_config=[{'rescue_robot': 4}],
                                 flags={'use_intention_map': True, 'use_shortest_path_to_receptacle_map': False}),
    # --- comparison variants (API completeness) ---
    'lifting_4-small_divider-history': dict(env_name='small_divider', robot_config=[{'lifting_robot': 4}],
                                            flags={'use_history_map': True}),
    'lifting_4-small_divider-binary': dict(env_name='small_divider', robot_config=[{'lifting_robot': 4}],
                                           flags={'use_intention_map': True, 'intention_map_encoding': 'binary'}),
    'lifting_4-large_empty-line': dict(env_name='large_empty', robot_config=[{'lifting_robot': 4}],
                                       flags={'use_intention_map': True, 'intention_map_encoding': 'line'}),
    'lifting_4-small_empty-circle': dict(env_name='small_empty', robot_config=[{'lifting_robot': 4}],
                                         flags={'use_intention_map': True, 'intention_map_encoding': 'circle'}),
    'lifting_4-small_divider-spatial': dict(env_name='small_divider', robot_config=[{'lifting_robot': 4}],
                                            flags={'use_intention_channels': True,
                                                   'intention_channel_encoding': 'spatial'}),
    'lifting_4-large_empty-nonspatial': dict(env_name='large_empty', robot_config=[{'lifting_robot': 4}],
                                             flags={'use_intention_channels': True,
                                                    'intention_channel_encoding': 'nonspatial'}),
    # use_distance_to_receptacle_map is an API flag no shipped config turns on (envs.py:2083-2084)
    'lifting_2_pushing_2-large_empty-all': dict(env_name='large_empty',
                                                robot_config=[{'lifting_robot': 2}, {'pushing_robot': 2}],
                                                flags={'use_distance_to_receptacle_map': True,
                                                       'use_history_map': True, 'use_intention_map': True,
                                                       'use_intention_channels': True}),
    # --- the reference's maze environments (envs.py:528-549, 577-592), config/experiments/ours/ ---
    'lifting_4-large_doors': dict(env_name='large_doors', robot_config=[{'lifting_robot': 4}],
                                  flags={'use_intention_map': True}, long_paths=True),
    'lifting_4-large_tunnels': dict(env_name='large_tunnels', robot_config=[{'lifting_robot': 4}],
                                    flags={'use_intention_map': True}, long_paths=True),
    'lifting_4-large_rooms': dict(env_name='large_rooms', robot_config=[{'lifting_robot': 4}],
                                  flags={'use_intention_map': True}, long_paths=True),
    'lifting_2_throwing_2-large_doors': dict(env_name='large_doors',
                                             robot_config=[{'lifting_robot': 2}, {'throwing_robot': 2}],
                                             flags={'use_intention_map': True}, long_paths=True),
    # config/experiments/comparisons/history_maps/lifting_4-large_rooms-history.yml
    'lifting_4-large_rooms-history': dict(env_name='large_rooms', robot_config=[{'lifting_robot': 4}],
                                          flags={'use_history_map': True}, long_paths=True),
}

MAZE_CONFIGS = ('lifting_4-large_doors', 'lifting_4-large_tunnels', 'lifting_4-large_rooms',
                'lifting_2_throwing_2-large_doors', 'lifting_4-large_rooms-history')

BASELINE_CONFIGS = ('lifting_1-small_empty', 'lifting_4-small_divider', 'pushing_4-large_empty',
                    'lifting_2_throwing_2-large_empty', 'rescue_4-small_empty')


def config_flags(name):
    cfg = CONFIGS[name]
    flags = dict(_BASE_FLAGS)
    flags.update(cfg['flags'])
    if any('rescue_robot' in g for g in cfg['robot_config']):  # utils.py:177-180
        flags['use_distance_to_receptacle_map'] = False
        flags['use_shortest_path_to_receptacle_map'] = False
    return flags


def num_channels(flags, num_robots):
    """Channel count of Mapper.get_state (envs.py:2068-2113)."""
    c = 1
    c += bool(flags['use_robot_map'])
    c += bool(flags['use_distance_to_receptacle_map'])
    c += bool(flags['use_shortest_path_to_receptacle_map'])
    c += bool(flags['use_shortest_path_map'])
    c += bool(flags['use_history_map'])
    c += bool(flags['use_intention_map'])
    if flags['use_intention_channels']:
        per = 1 if flags['intention_channel_encoding'] == 'spatial' else 2
        c += per * (num_robots - 1)
    return c


def pixel_center_positions(H, W):
    """Mapper.pixel_indices_to_position over the whole grid (envs.py:2399-2403), fp64."""
    ii, jj = np.meshgrid(np.arange(H), np.arange(W), indexing='ij')
    x = ((jj + 0.5) - W / 2) / K.LOCAL_MAP_PIXELS_PER_METER
    y = (H / 2 - (ii + 0.5)) / K.LOCAL_MAP_PIXELS_PER_METER
    return x, y


def _obstacles(env_name, room_length, room_width, rs):
    """Boxes of VectorEnv._get_obstacles (envs.py:515-571), the wall / divider corners
    (envs.py:589-647) and the robot / cube spawn bounds.

    Returns (boxes [(x, y, x_len, y_len)], divider_corners [(x, y, heading_deg)], robot_bounds,
    cube_bounds).  The room corners (envs.py:573-587) are added by make_scene.  The random draws
    follow the reference's order (room_random_state: one uniform per offset)."""
    wall_thickness = 1.4
    boxes = []
    for x, y, length, width in [
            (-room_length / 2 - wall_thickness / 2, 0, wall_thickness, room_width),
            (room_length / 2 + wall_thickness / 2, 0, wall_thickness, room_width),
            (0, -room_width / 2 - wall_thickness / 2, room_length + 2 * wall_thickness, wall_thickness),
            (0, room_width / 2 + wall_thickness / 2, room_length + 2 * wall_thickness, wall_thickness)]:
        boxes.append((x, y, length, width))
    dividers = []  # (x, y, x_len, y_len, snap_y or None)
    spawn_bounds = cube_bounds = None
    if env_name in ('small_divider', 'small_divider_norand'):
        x_offset = rs.uniform(-0.1, 0.1) if env_name == 'small_divider' else 0.0
        divider_width, opening_width = 0.05, 0.16
        dividers.append((x_offset, 0.0, divider_width, room_width - 2 * opening_width, None))
        spawn_bounds = (x_offset + divider_width / 2, None, None, None)
        cube_bounds = (None, x_offset - divider_width / 2, None, None)
    elif env_name in ('large_doors', 'large_doors_norand', 'large_tunnels', 'large_tunnels_norand'):
        tunnel_length = 0.05 if env_name.startswith('large_doors') else 0.25
        x_offset = y_offset = 0.0
        if env_name == 'large_doors':
            x_offset, y_offset = rs.uniform(-0.05, 0.05), rs.uniform(-0.1, 0.1)
        elif env_name == 'large_tunnels':
            x_offset, y_offset = rs.uniform(-0.05, 0.05), rs.uniform(-0.05, 0.05)
        tunnel_width = 0.18  # add_tunnels (envs.py:530-540)
        tunnel_x = (room_length + tunnel_width) / 6 + x_offset
        outer_divider_len = room_length / 2 - tunnel_x - tunnel_width / 2
        divider_x = room_length / 2 - outer_divider_len / 2
        middle_divider_len = 2 * (tunnel_x - tunnel_width / 2)
        dividers.append((-divider_x, y_offset, outer_divider_len, tunnel_length, None))
        dividers.append((0.0, y_offset, middle_divider_len, tunnel_length, None))
        dividers.append((divider_x, y_offset, outer_divider_len, tunnel_length, None))
        spawn_bounds = (None, None, y_offset + tunnel_length / 2, None)
        cube_bounds = (None, None, None, y_offset - tunnel_length / 2)
    elif env_name in ('large_rooms', 'large_rooms_norand'):
        x_offset = y_offset = 0.0
        if env_name == 'large_rooms':
            x_offset, y_offset = rs.uniform(-0.05, 0.05), rs.uniform(-0.05, 0.05)
        divider_width, opening_width = 0.05, 0.18  # add_rooms (envs.py:542-551)
        divider_len = room_width / 2 - opening_width - divider_width / 2
        top_divider_len = divider_len - y_offset
        bot_divider_len = divider_len + y_offset
        top_divider_y = room_width / 2 - opening_width - top_divider_len / 2
        bot_divider_y = -room_width / 2 + opening_width + bot_divider_len / 2
        dividers.append((0.0, y_offset, room_length - 2 * opening_width, divider_width, None))
        dividers.append((x_offset, top_divider_y, divider_width, top_divider_len, y_offset + divider_width / 2))
        dividers.append((x_offset, bot_divider_y, divider_width, bot_divider_len, y_offset - divider_width / 2))
    elif env_name not in ('small_empty', 'large_empty'):
        raise ValueError('unknown env_name %r' % env_name)
    corners = []
    for (x, y, length, width, snap_y) in dividers:  # corners between walls and dividers (envs.py:610-641)
        boxes.append((x, y, length, width))
        pos = None
        if math.isclose(x - length / 2, -room_length / 2):
            pos, hd = [(-room_length / 2, y - width / 2), (-room_length / 2, y + width / 2)], [0, 90]
        elif math.isclose(x + length / 2, room_length / 2):
            pos, hd = [(room_length / 2, y - width / 2), (room_length / 2, y + width / 2)], [-90, 180]
        elif math.isclose(y - width / 2, -room_width / 2):
            pos, hd = [(x - length / 2, -room_width / 2), (x + length / 2, -room_width / 2)], [180, 90]
        elif math.isclose(y + width / 2, room_width / 2):
            pos, hd = [(x - length / 2, room_width / 2), (x + length / 2, room_width / 2)], [-90, 0]
        elif snap_y is not None:
            pos = [(x - length / 2, snap_y), (x + length / 2, snap_y)]
            hd = [-90, 0] if snap_y > y else [180, 90]
        if pos is not None:
            corners.extend((px, py, h) for (px, py), h in zip(pos, hd))
    return boxes, corners, spawn_bounds, cube_bounds


def _corner_mask(X, Y, cx, cy, heading_deg, w=0.1006834873):
    """A rounded corner obstacle at corner point (cx, cy): the w x w square on the diagonal at
    heading - 45 degrees (envs.py:583-586, 637-640) minus the quarter disk of radius w centred on
    its far corner (the corner body's curved face)."""
    a = math.radians(heading_deg - 45)
    sx, sy = math.copysign(1, round(math.cos(a), 12)), math.copysign(1, round(math.sin(a), 12))
    in_sq = (np.abs(X - cx) <= w) & (np.abs(Y - cy) <= w) & ((X - cx) * sx >= 0) & ((Y - cy) * sy >= 0)
    ox, oy = cx + sx * w, cy + sy * w
    return in_sq & ((X - ox) ** 2 + (Y - oy) ** 2 > w * w)


def _random_position(rs, room_length, room_width, padding, bounds=None):
    """VectorEnv._get_random_position (envs.py:700-716)."""
    low_x, high_x = -room_length / 2 + padding, room_length / 2 - padding
    low_y, high_y = -room_width / 2 + padding, room_width / 2 - padding
    if bounds is not None:
        x_min, x_max, y_min, y_max = bounds
        if x_min is not None:
            low_x = x_min + padding
        if x_max is not None:
            high_x = x_max - padding
        if y_min is not None:
            low_y = y_min + padding
        if y_max is not None:
            high_y = y_max - padding
    px, py = rs.uniform((low_x, low_y), (high_x, high_y))
    return float(px), float(py)


def make_scene(config_name, env_idx, seed_base=1234, observe_all=False):
    """One env's observation-path inputs.

    Returns a dict:
      env_name, room_length, room_width, flags, robot_config, H, W,
      receptacle_position (x, y, 0) or None,
      robots: list of dicts {type, cls, group_index, position (x,y,0), heading, lift_state, idle,
                             waypoint_positions [(x,y,0)...], waypoint_index, target_ee (x,y,0)},
      occupancy: u8 [A, H, W]  (per agent, OccupancyMap.occupancy_map after update)
      overhead: f32 [A, H, W]  (per agent, Mapper.global_overhead_map_without_robots)
      obstacle_mask: bool [H, W] (ground truth, for the point cloud of the golden generator)
    """
    return _scene(config_name, CONFIGS[config_name], config_flags(config_name), env_idx, seed_base, observe_all)


def reference_config_scene(row, env_idx, seed_base=4321, observe_all=False):
    """A scene for one reference experiment config as tests/golden/reference_configs.json holds it
    (config/**/*.yml: env_name, robot_config, the state-representation flags): the obstacle layout
    of its env_name (the maze layouts' longer paths included), its robots, its flags."""
    maze = row['env_name'] in ('large_doors', 'large_tunnels', 'large_rooms')
    cfg = dict(env_name=row['env_name'], robot_config=row['robot_config'], long_paths=maze)
    flags = dict(_BASE_FLAGS)
    flags.update(row['flags'])
    return _scene(row['config'], cfg, flags, env_idx, seed_base, observe_all)


def _scene(config_name, cfg, flags, env_idx, seed_base, observe_all):
    rs = np.random.RandomState(seed_base + env_idx)
    room_length, room_width, num_cubes = K.room_dims(cfg['env_name'])
    H, W = K.padded_room_shape(room_width, room_length)
    is_rescue = any('rescue_robot' in g for g in cfg['robot_config'])
    receptacle = None if is_rescue else (room_length / 2 - K.RECEPTACLE_WIDTH / 2,
                                         room_width / 2 - K.RECEPTACLE_WIDTH / 2, 0)  # envs.py:150-151

    boxes, div_corners, spawn_bounds, cube_bounds = _obstacles(cfg['env_name'], room_length, room_width, rs)
    maze = cfg.get('long_paths', False)
    X, Y = pixel_center_positions(H, W)
    obstacle = np.zeros((H, W), dtype=bool)
    for (bx, by, bl, bw) in boxes:
        obstacle |= (np.abs(X - bx) <= bl / 2) & (np.abs(Y - by) <= bw / 2)
    # Rounded room corners (envs.py:573-587): a w x w square minus a quarter disk.
    w = 0.1006834873
    for (cx, cy) in [(-room_length / 2, room_width / 2), (room_length / 2, room_width / 2),
                     (room_length / 2, -room_width / 2), (-room_length / 2, -room_width / 2)]:
        if receptacle is not None and math.hypot(cx - receptacle[0], cy - receptacle[1]) <= \
                (1 + 1e-6) * (K.RECEPTACLE_WIDTH / 2) * math.sqrt(2):
            continue
        sx, sy = -math.copysign(1, cx), -math.copysign(1, cy)
        in_sq = (np.abs(X - cx) <= w) & (np.abs(Y - cy) <= w) & ((X - cx) * sx >= 0) & ((Y - cy) * sy >= 0)
        ox, oy = cx + sx * w, cy + sy * w
        obstacle |= in_sq & ((X - ox) ** 2 + (Y - oy) ** 2 > w * w)
    for (cx, cy, hd) in div_corners:
        obstacle |= _corner_mask(X, Y, cx, cy, hd)

    in_room = (np.abs(X) <= room_length / 2) & (np.abs(Y) <= room_width / 2)
    seg = np.where(in_room, K.SEG_VALUES['floor'], K.SEG_VALUES['obstacle']).astype(np.float32)
    seg[obstacle] = K.SEG_VALUES['obstacle']
    if receptacle is not None:
        rec = (np.abs(X - receptacle[0]) <= K.RECEPTACLE_WIDTH / 2) & (np.abs(Y - receptacle[1]) <= K.RECEPTACLE_WIDTH / 2)
        seg[rec & in_room & ~obstacle] = K.SEG_VALUES['receptacle']
    for _ in range(num_cubes):
        # (the BASELINE configs' scenes predate the cube spawn bounds; the maze configs use them)
        px, py = _random_position(rs, room_length, room_width, K.CUBE_WIDTH / 2, cube_bounds if maze else None)
        cube = (np.abs(X - px) <= K.CUBE_WIDTH / 2) & (np.abs(Y - py) <= K.CUBE_WIDTH / 2)
        seg[cube & in_room & ~obstacle] = K.SEG_VALUES['cube']

    robots = []
    for group_index, g in enumerate(cfg['robot_config']):
        rtype, count = next(iter(g.items()))
        geom = K.ROBOT_GEOM[rtype]
        for _ in range(count):
            px, py = _random_position(rs, room_length, room_width, geom['RADIUS'], spawn_bounds)
            heading = float(rs.uniform(-math.pi, math.pi))
            # maze configs: longer movement paths (doors / tunnels / rooms need more waypoints)
            n_wp = int(rs.randint(2, 6)) if not maze else int(rs.randint(4, 12))
            wps = [(px, py, 0)]
            for _ in range(n_wp - 1):
                wx, wy = _random_position(rs, room_length, room_width, geom['RADIUS'])
                wps.append((wx, wy, 0))
            tx, ty = _random_position(rs, room_length, room_width, 0.0)
            robots.append({
                'type': rtype, 'cls': K.ROBOT_TYPES.index(rtype), 'group_index': group_index,
                'position': (px, py, 0), 'heading': heading,
                'lift_state': 'lifting' if (rtype == 'lifting_robot' and rs.rand() < 0.5) else 'ready',
                'idle': bool(len(robots) == 0 or rs.rand() < 0.15),
                'waypoint_positions': wps,
                'waypoint_index': int(rs.randint(1, n_wp)),
                'target_ee': (tx, ty, 0),
            })

    # Per-agent observed maps (partial observation: a disk around the agent plus a random
    # earlier viewpoint), values as Mapper.update writes them (envs.py:2057-2066).
    A = len(robots)
    occupancy = np.zeros((A, H, W), dtype=np.uint8)
    overhead = np.zeros((A, H, W), dtype=np.float32)
    for a, r in enumerate(robots):
        if observe_all:
            seen = np.ones((H, W), dtype=bool)
        else:
            seen = np.zeros((H, W), dtype=bool)
            for (vx, vy) in [r['position'][:2], _random_position(rs, room_length, room_width, 0.0)]:
                rad = rs.uniform(0.35, 1.2)
                seen |= (X - vx) ** 2 + (Y - vy) ** 2 <= rad * rad
        overhead[a][seen] = seg[seen]
        occupancy[a][seen & (seg == K.SEG_VALUES['obstacle'])] = 1

    return {
        'config': config_name, 'env_name': cfg['env_name'], 'room_length': room_length,
        'room_width': room_width, 'flags': flags, 'robot_config': cfg['robot_config'], 'H': H, 'W': W,
        'receptacle_position': receptacle, 'robots': robots,
        'occupancy': occupancy, 'overhead': overhead, 'seg_truth': seg,
        'rotate_rounding': 'fma',  # the synthetic scenes render with the fused form
    }


def never_acted(scene, robots=None):
    """A copy of `scene` whose robots `robots` (all if None) have not acted yet: the state
    Robot.__init__ / Robot.reset leave until the robot's first store_new_action (envs.py:828-832,
    958-963; RobotController.__init__ 1373-1376) -- controller idle, waypoint_positions,
    target_end_effector_position and waypoint_index None, LiftingRobot.lift_state 'ready'
    (envs.py:1175).  All robots: what VectorEnv.reset() renders (envs.py:214-222)."""
    out = dict(scene)
    out['robots'] = [dict(r) for r in scene['robots']]
    for k, r in enumerate(out['robots']):
        if robots is None or k in robots:
            r.update(idle=True, waypoint_positions=None, waypoint_index=None, target_ee=None)
            if r['type'] == 'lifting_robot':
                r['lift_state'] = 'ready'
    return out


def intention_path(robot):
    """RobotController.get_intention_path (envs.py:1475-1476)."""
    idx = robot['waypoint_index']
    return [robot['position']] + list(robot['waypoint_positions'][idx:-1]) + [robot['target_ee']]


def history_path(robot):
    """RobotController.get_history_path (envs.py:1478-1479)."""
    idx = robot['waypoint_index']
    return list(robot['waypoint_positions'][:idx]) + [robot['position']]


# Body ids of the synthetic scenes' segmentation masks (pybullet getCameraImage seg buffer):
# 0 = floor plane, obstacles 1..2, cubes 3..4, receptacle 99, robot k = 10 + k, -1 = background.
SEG_IDS = {'min_obstacle': 1, 'max_obstacle': 2, 'min_cube': 3, 'max_cube': 4, 'receptacle': 99}


def camera_images(scene, agent, kind='forward', seed=0):
    """A synthetic pybullet-like frame of robot `agent`'s camera (Camera.capture_image input,
    envs.py:1927-1930): (depth_buffer float32 [Hc, Wc] in [0, 1], seg_raw int32 [Hc, Wc]).

    Rays of the camera model hit a floor whose pixels carry the scene's classes at class heights
    (walls 0.1 m, cubes 0.044 m, robots 0.07 m), plus tiny depth noise so that no two points share
    a z value (the reference's argsort breaks z ties in an unspecified order)."""
    from .camera import CAMERAS
    spec = CAMERAS[kind]
    rs = np.random.RandomState(seed)
    r = scene['robots'][agent]
    pos, tgt, up = np.array(spec.params(r['position'][0], r['position'][1], r['heading'])).reshape(3, 3)
    principal = tgt - pos
    principal /= np.linalg.norm(principal)
    up = up - np.dot(up, principal) * principal
    up /= np.linalg.norm(up)
    right = np.cross(principal, up)
    right /= np.linalg.norm(right)
    Hc, Wc = spec.height_px, spec.width_px
    px = spec.cx2 * (np.arange(Wc) / Wc - 0.5)
    py = spec.cy2 * (0.5 - (np.arange(Hc) + 1) / Hc)
    d = principal[None, None, :] + px[None, :, None] * right[None, None, :] + py[:, None, None] * up[None, None, :]
    H, W = scene['H'], scene['W']
    seg_truth = scene['seg_truth']

    def classify(x, y):
        pi = np.clip(np.floor(H / 2 - y * K.LOCAL_MAP_PIXELS_PER_METER).astype(np.int64), 0, H - 1)
        pj = np.clip(np.floor(W / 2 + x * K.LOCAL_MAP_PIXELS_PER_METER).astype(np.int64), 0, W - 1)
        s = seg_truth[pi, pj]
        raw = np.full(x.shape, -1, dtype=np.int32)
        raw[s == K.SEG_VALUES['floor']] = 0
        raw[s == K.SEG_VALUES['obstacle']] = 1 + (pi[s == K.SEG_VALUES['obstacle']] % 2)
        raw[s == K.SEG_VALUES['receptacle']] = SEG_IDS['receptacle']
        raw[s == K.SEG_VALUES['cube']] = 3 + (pj[s == K.SEG_VALUES['cube']] % 2)
        for k, o in enumerate(scene['robots']):
            if k != agent:
                raw[(x - o['position'][0]) ** 2 + (y - o['position'][1]) ** 2 <= 0.05 ** 2] = 10 + k
        return raw

    height = {-1: 0.0, 0: 0.0, 1: 0.1, 2: 0.1, 3: 0.044, 4: 0.044, SEG_IDS['receptacle']: 0.001}
    down = d[..., 2] < -1e-9
    depth = np.full((Hc, Wc), float(spec.far))
    t0 = np.where(down, -pos[2] / np.where(down, d[..., 2], -1.0), np.inf)
    raw = classify(pos[0] + t0 * d[..., 0], pos[1] + t0 * d[..., 1])
    h = np.vectorize(lambda v: height.get(int(v), 0.07))(raw)
    t = np.where(down, (h - pos[2]) / np.where(down, d[..., 2], -1.0), np.inf)
    t = np.where(t > 0, t, t0)
    depth = np.where(down, np.minimum(t, spec.far), spec.far)
    raw = np.where(down & (t <= spec.far), raw, -1).astype(np.int32)
    depth = np.maximum(depth, spec.near)
    db = (spec.far - spec.far * spec.near / depth) / (spec.far - spec.near)
    db = np.clip(db + rs.uniform(-2e-6, 2e-6, db.shape), 0.0, 1.0).astype(np.float32)
    return db, raw
