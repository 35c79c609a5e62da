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
