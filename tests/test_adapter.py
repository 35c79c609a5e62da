"""CPU: the reference-object adapter reads a VectorEnv-shaped object into the same device
descriptors as the scene it was built from (objects carry the reference's attribute names)."""
from types import SimpleNamespace

import numpy as np

import json

import pytest

import goldens as G
from simaps import batch, reference_adapter, synthetic


class _Robot:
    def __init__(self, r, occ, ovh):
        self.group_index = r['group_index']
        self._pos, self._h = r['position'], r['heading']
        self.waypoint_positions = None if r['waypoint_positions'] is None else list(r['waypoint_positions'])
        self.target_end_effector_position = r['target_ee']
        self.controller = SimpleNamespace(waypoint_index=r['waypoint_index'], state='idle' if r['idle'] else 'moving')
        self.mapper = SimpleNamespace(global_overhead_map_without_robots=ovh,
                                      global_occupancy_map=SimpleNamespace(occupancy_map=occ))
        self.awaiting_new_action = not r['idle']
        if r['type'] == 'lifting_robot':
            self.lift_state = r['lift_state']

    def get_position(self):
        return self._pos

    def get_heading(self):
        return self._h

    def is_idle(self):
        return self.controller.state == 'idle'


CLASSES = {c: type(c, (_Robot,), {}) for c in reference_adapter.ROBOT_TYPE_BY_CLASS}
BY_TYPE = {v: CLASSES[k] for k, v in reference_adapter.ROBOT_TYPE_BY_CLASS.items()}


def _fake_env(scene):
    env = SimpleNamespace(**scene['flags'], room_length=scene['room_length'], room_width=scene['room_width'],
                          robot_config=scene['robot_config'])
    if scene['receptacle_position'] is not None:
        env.receptacle_position = scene['receptacle_position']
    env.robots = [BY_TYPE[r['type']](r, scene['occupancy'][k], scene['overhead'][k]) for k, r in enumerate(scene['robots'])]
    return env


def test_scene_from_env_round_trip():
    for cfg in ('lifting_4-small_divider', 'lifting_2_throwing_2-large_empty', 'rescue_4-small_empty',
                'lifting_2_pushing_2-large_empty-all'):
        s = synthetic.make_scene(cfg, 3)
        got = reference_adapter.scene_from_env(_fake_env(s))
        agents = [(0, a) for a in range(len(s['robots']))]
        for x, y in zip(batch.pack_descriptors([s], agents), batch.pack_descriptors([got], agents)):
            assert x.tobytes() == y.tobytes()
        assert np.array_equal(got['occupancy'], s['occupancy']) and np.array_equal(got['overhead'], s['overhead'])
        assert got['flags'] == s['flags'] and (got['H'], got['W']) == (s['H'], s['W'])
        assert reference_adapter.awaiting_flags(_fake_env(s)) == [not r['idle'] for r in s['robots']]


def _pack_per_robot(scenes, agents):
    """The straightforward per-robot, per-field packing (batch.pack_descriptors before it was made
    column-wise): the layout every kernel reads, field by field."""
    from simaps import _lib
    robots = np.zeros(sum(len(s['robots']) for s in scenes), dtype=_lib.ROBOT_DTYPE)
    envs = np.zeros(len(scenes), dtype=_lib.ENV_DTYPE)
    paths, k = [], 0
    for e, s in enumerate(scenes):
        envs[e]['robot_off'], envs[e]['num_robots'] = k, len(s['robots'])
        rec = s['receptacle_position']
        envs[e]['has_receptacle'] = rec is not None
        if rec is not None:
            envs[e]['receptacle_x'], envs[e]['receptacle_y'] = rec[0], rec[1]
        for r in s['robots']:
            R = robots[k]
            R['x'], R['y'], R['heading'] = r['position'][0], r['position'][1], r['heading']
            R['target_x'], R['target_y'] = r['target_ee'][0], r['target_ee'][1]
            R['type'], R['group_index'] = _lib.TYPE_IDS[r['type']], r['group_index']
            R['lifting'], R['idle'] = int(r.get('lift_state') == 'lifting'), int(bool(r['idle']))
            idx = r['waypoint_index']
            for name, pts in (('intention', [r['position']] + list(r['waypoint_positions'][idx:-1]) + [r['target_ee']]),
                              ('history', (list(r['waypoint_positions'][:idx]) + [r['position']])[::-1])):
                R[name + '_off'], R[name + '_len'] = len(paths), len(pts)
                paths.extend((float(p[0]), float(p[1])) for p in pts)
            k += 1
    ag = np.zeros(len(agents), dtype=_lib.AGENT_DTYPE)
    for n, (e, a) in enumerate(agents):
        ag[n]['env'], ag[n]['robot'], ag[n]['map_slot'] = e, a, n
    return robots, envs, ag, np.array(paths if paths else [(0.0, 0.0)], dtype=np.float64).reshape(-1, 2)


def test_pack_descriptors_bytes_match_per_robot_packing():
    """The column-wise packer writes byte-identical C structs (robots, envs, agents, path points)."""
    for cfg in ('lifting_4-small_divider', 'lifting_2_throwing_2-large_empty', 'rescue_4-small_empty',
                'lifting_2_pushing_2-large_empty-all', 'lifting_4-large_rooms-history'):
        scenes = [synthetic.make_scene(cfg, 70 + e) for e in range(5)]
        agents = [(e, a) for e, s in enumerate(scenes) for a in range(len(s['robots']))][::-1][:-2]
        for got, want in zip(batch.pack_descriptors(scenes, agents), _pack_per_robot(scenes, agents)):
            assert got.dtype == want.dtype and got.tobytes() == want.tobytes(), cfg


def test_scene_from_env_reset_and_not_yet_acted_robots():
    """VectorEnv.reset() state (envs.py:214-222): every robot idle with waypoint_positions /
    target_end_effector_position / controller.waypoint_index None (envs.py:828-832, 958-963,
    1373-1376) -- and the mixed state after it.  The adapter passes None through and the packer
    gives those robots no paths."""
    base = synthetic.make_scene('lifting_4-small_divider', 5)
    for sc in (synthetic.never_acted(base), synthetic.never_acted(base, robots=[1, 2, 3])):
        got = reference_adapter.scene_from_env(_fake_env(sc))
        assert [r['target_ee'] for r in got['robots']] == [r['target_ee'] for r in sc['robots']]
        agents = [(0, a) for a in range(4)]
        x, y = batch.pack_descriptors([sc], agents), batch.pack_descriptors([got], agents)
        assert all(p.tobytes() == q.tobytes() for p, q in zip(x, y))
        rob = x[0]
        never = np.array([r['waypoint_positions'] is None for r in sc['robots']])
        assert (rob['idle'][never] == 1).all()
        assert (rob['intention_len'][never] == 0).all() and (rob['history_len'][never] == 0).all()
        assert (rob['target_x'][never] == 0).all()


def test_pack_rejects_moving_robot_without_path():
    sc = synthetic.never_acted(synthetic.make_scene('lifting_4-small_divider', 5), robots=[2])
    sc['robots'][2]['idle'] = False
    with pytest.raises(ValueError):
        batch.pack_descriptors([sc], [(0, 0)])


RESET_FILES = [f for f in G.scene_files() if '/scene_reset_' in f or '/scene_rot-' in f]


@pytest.mark.parametrize('path', RESET_FILES, ids=[f.rsplit('/', 1)[1] for f in RESET_FILES])
def test_adapter_on_reference_objects_matches_fixture(path):
    """make_goldens.py ran reference_adapter.scene_from_env on the reference's OWN LiftingRobot /
    RobotController objects (reset and never-acted robots included) and recorded what it returned:
    that descriptor packs byte-identically to the fixture's scene, and in the reset env every robot
    packs as idle with no paths."""
    z = G.load(path.rsplit('/', 1)[1])
    e = 0
    while 'e%d_scene' % e in z.files:
        want = json.loads(str(z['e%d_scene' % e]))
        got = json.loads(str(z['e%d_adapter' % e]))
        assert got['rotate_rounding'] == want['rotate_rounding']
        for gr, wr in zip(got['robots'], want['robots']):
            for k in ('type', 'group_index', 'idle', 'waypoint_index', 'heading'):
                assert gr[k] == wr[k], k
            if wr['type'] == 'lifting_robot':  # (only LiftingRobot has a lift_state, envs.py:1175)
                assert gr['lift_state'] == wr['lift_state']
            assert gr['position'][:2] == wr['position'][:2]
            assert (gr['target_ee'] is None) == (wr['target_ee'] is None)
            assert (gr['waypoint_positions'] is None) == (wr['waypoint_positions'] is None)
        agents = [(0, a) for a in range(len(want['robots']))]
        for p, q in zip(batch.pack_descriptors([want], agents), batch.pack_descriptors([got], agents)):
            assert p.tobytes() == q.tobytes()
        if '/scene_reset_' in path and e == 0:
            rob = batch.pack_descriptors([got], agents)[0]
            assert (rob['idle'] == 1).all() and (rob['intention_len'] == 0).all()
        e += 1


@pytest.mark.parametrize('cfg', ['lifting_4-small_divider', 'lifting_2_throwing_2-large_empty', 'rescue_4-small_empty',
                                 'lifting_4-large_rooms-history', 'lifting_4-large_doors'])
def test_native_pack_robots_matches_scene_packing(cfg):
    """simaps_pack_robots (the drop-in's array fast path, host C++) writes the same robot records and
    the same intention / history path points as pack_descriptors -- only the path offsets differ
    (fixed stride 2 * SIMAPS_MAX_PATH per robot) -- including robots that never acted."""
    from simaps import _lib
    scenes = [synthetic.make_scene(cfg, 40 + e) for e in range(4)]
    scenes[1] = synthetic.never_acted(scenes[1])
    scenes[2] = synthetic.never_acted(scenes[2], robots=[1, 2])
    agents = [(e, a) for e, s in enumerate(scenes) for a in range(len(s['robots']))]
    want_r, _, _, want_p = batch.pack_descriptors(scenes, agents)
    d = batch.descriptor_arrays(scenes)
    R = len(want_r)
    P = _lib.MAX_PATH
    tg = np.array([(_lib.TYPE_IDS[r['type']], r['group_index']) for s in scenes for r in s['robots']], np.int32)
    flags = d['idle'].astype(np.int32) | (d['lifting'].astype(np.int32) << 1)
    got_r = np.zeros(R, _lib.ROBOT_DTYPE)
    got_p = np.zeros((R * 2 * P, 2))
    K = d['waypoints'].shape[1]
    assert _lib.lib.simaps_pack_robots(R, d['pose'].ctypes.data, d['target'].ctypes.data, flags.ctypes.data,
                                       tg.ctypes.data, d['waypoints'].ctypes.data, K, d['wp_count'].ctypes.data,
                                       d['wp_index'].ctypes.data, got_r.ctypes.data, got_p.ctypes.data) == 0
    for f in _lib.ROBOT_DTYPE.names:
        if f.endswith('_off'):
            continue
        assert np.array_equal(got_r[f], want_r[f]), f
    for k in range(R):
        for name in ('intention', 'history'):
            n = want_r[name + '_len'][k]
            a = want_p[want_r[name + '_off'][k]:][:n]
            b = got_p[got_r[name + '_off'][k]:][:n]
            assert a.tobytes() == b.tobytes(), (k, name)


def test_native_pack_robots_rejects_bad_rows():
    from simaps import _lib
    scenes = [synthetic.make_scene('lifting_4-small_divider', 1)]
    d = batch.descriptor_arrays(scenes)
    tg = np.zeros((4, 2), np.int32)
    out_r = np.zeros(4, _lib.ROBOT_DTYPE)
    out_p = np.zeros((4 * 2 * _lib.MAX_PATH, 2))

    def pack(flags, cnt, idx, wps):
        return _lib.lib.simaps_pack_robots(4, d['pose'].ctypes.data, d['target'].ctypes.data, flags.ctypes.data,
                                           tg.ctypes.data, wps.ctypes.data, wps.shape[1], cnt.ctypes.data,
                                           idx.ctypes.data, out_r.ctypes.data, out_p.ctypes.data)
    moving = np.zeros(4, np.int32)
    cnt = d['wp_count'].copy()
    cnt[2] = -1  # None paths on a moving robot
    assert pack(moving, cnt, d['wp_index'], d['waypoints']) == _lib.EINVAL
    long_w = np.zeros((4, 20, 2))
    assert pack(moving, np.full(4, 20, np.int32), np.ones(4, np.int32), long_w) == _lib.EUNSUPPORTED
