"""CPU: the reference-object adapter reads a VectorEnv-shaped object into the same device
descriptors as the scene it was built from (objects carry the reference's attribute names)."""
from types import SimpleNamespace

import numpy as np

from simaps import batch, reference_adapter, synthetic


class _Robot:
    def __init__(self, r, occ, ovh):
        self.group_index = r['group_index']
        self._pos, self._h = r['position'], r['heading']
        self.waypoint_positions = list(r['waypoint_positions'])
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
