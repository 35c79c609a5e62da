"""Host side of the mixed-configuration launch (simaps_get_state_mixed): the plan MixedStateBatch
hands the kernel, and the C ABI's argument checks (which return before any HIP call)."""
import ctypes

import numpy as np
import pytest

from simaps import _lib, batch, synthetic

MIX = [('lifting_4-small_divider', 0), ('pushing_4-large_empty', 1), ('lifting_4-small_divider', 2),
       ('rescue_4-small_empty', 3), ('lifting_4-large_empty-nonspatial', 4), ('lifting_2_throwing_2-large_doors', 5)]


def _scenes(mix=MIX):
    return [synthetic.make_scene(c, e) for c, e in mix]


def test_plan_groups_offsets_and_channels():
    sc = _scenes()
    p = batch.plan_mixed(sc, 'chw')
    # robot classes and the obstacle layout are per scene: pushing_4-large_empty and
    # lifting_2_throwing_2-large_doors share a configuration (grid, room, flags)
    assert p['cfg_of_env'] == [0, 1, 0, 2, 3, 1]
    assert len(p['cfgs']) == 4
    agents = [(e, a) for e, s in enumerate(sc) for a in range(len(s['robots']))]
    assert p['agents'] == agents
    assert list(p['agent_cfg']) == [p['cfg_of_env'][e] for e, _ in agents]
    hw = [sc[e]['H'] * sc[e]['W'] for e, _ in agents]
    assert list(p['map_off']) == list(np.cumsum([0] + hw[:-1]))
    assert p['map_numel'] == sum(hw)
    for k, c in enumerate(p['cfgs']):
        s0 = sc[p['cfg_of_env'].index(k)]
        assert (c.H, c.W, c.layout_chw) == (s0['H'], s0['W'], 1)
        assert p['channels'][k] == _lib.lib.simaps_num_channels(c, len(s0['robots']))
    per = [96 * 96 * p['channels'][k] for k in p['agent_cfg']]
    assert list(p['out_off']) == list(np.cumsum([0] + per[:-1])) and p['out_numel'] == sum(per)
    assert p['num_robots'][p['cfg_of_env'][4]] == 4  # intention channels: the robot count goes to the ABI
    assert p['num_robots'][0] == 0


def test_plan_splits_rotate_rounding_and_layout():
    sc = _scenes(MIX[:1]) + [dict(synthetic.make_scene('lifting_4-small_divider', 9), rotate_rounding='plain')]
    p = batch.plan_mixed(sc, 'hwc')
    assert p['cfg_of_env'] == [0, 1] and [c.rotate_rounding for c in p['cfgs']] == [0, 1]
    assert all(c.layout_chw == 0 for c in p['cfgs'])


def test_plan_limits():
    cfgs = ['lifting_1-small_empty', 'lifting_4-small_divider', 'pushing_4-large_empty', 'rescue_4-small_empty',
            'lifting_4-small_divider-history', 'lifting_4-large_empty-line', 'lifting_4-small_empty-circle',
            'lifting_4-small_divider-spatial', 'lifting_4-large_empty-nonspatial']  # 9 distinct configurations
    assert len(batch.plan_mixed(_scenes([(c, e) for e, c in enumerate(cfgs[:8])]))['cfgs']) == _lib.MAX_MIXED
    with pytest.raises(ValueError, match='at most 8 configurations'):
        batch.plan_mixed(_scenes([(c, e) for e, c in enumerate(cfgs)]))
    # with intention channels, each robot count is its own table entry (its own channel count)
    a = synthetic.make_scene('lifting_4-large_empty-nonspatial', 0)
    b = synthetic.make_scene('lifting_4-large_empty-nonspatial', 1)
    b = dict(b, robots=b['robots'][:3], occupancy=b['occupancy'][:3], overhead=b['overhead'][:3])
    p = batch.plan_mixed([a, b, a])
    assert p['cfg_of_env'] == [0, 1, 0] and p['num_robots'] == [4, 3]
    assert p['channels'][0] == p['channels'][1] + 2  # nonspatial: 2 channels per other robot
    # without them, robot counts share an entry
    c = synthetic.make_scene('lifting_4-small_divider', 0)
    d = synthetic.make_scene('lifting_4-small_divider', 1)
    d = dict(d, robots=d['robots'][:2], occupancy=d['occupancy'][:2], overhead=d['overhead'][:2])
    assert batch.plan_mixed([c, d])['cfg_of_env'] == [0, 0]


def test_mixed_needs_a_gpu_device():
    with pytest.raises(ValueError, match='no CPU path'):
        batch.MixedStateBatch(_scenes(MIX[:2]), device='cpu')


def test_abi_argument_checks():
    L = _lib.lib
    p = batch.plan_mixed(_scenes(), 'chw')
    cfgs = (_lib.Config * len(p['cfgs']))(*p['cfgs'])
    nrs = np.asarray(p['num_robots'], dtype=np.int32)
    null = [None] * 11

    def call(cf, nr, n, N, bufs=null):
        return L.simaps_get_state_mixed(cf, nr, n, N, *bufs)

    assert call(cfgs, nrs.ctypes.data, 0, 1) == _lib.EINVAL
    assert call(cfgs, nrs.ctypes.data, _lib.MAX_MIXED + 1, 1) == _lib.EINVAL
    assert call(None, nrs.ctypes.data, 1, 1) == _lib.EINVAL
    k = p['cfg_of_env'][4]  # intention channels: a robot count is required
    bad = nrs.copy()
    bad[k] = 0
    assert call(cfgs, bad.ctypes.data, len(p['cfgs']), 1) == _lib.EINVAL
    assert 'intention channels' in L.simaps_last_error().decode()
    assert call(cfgs, nrs.ctypes.data, len(p['cfgs']), -1) == _lib.EINVAL
    assert call(cfgs, nrs.ctypes.data, len(p['cfgs']), 0) == 0  # nothing to do: no launch
    assert call(cfgs, nrs.ctypes.data, len(p['cfgs']), 4) == _lib.EINVAL  # NULL buffers
    assert 'NULL' in L.simaps_last_error().decode()
    broken = (_lib.Config * 1)(p['cfgs'][0])
    broken[0].H = 0
    assert call(broken, None, 1, 1) == _lib.EINVAL
    assert ctypes.sizeof(_lib.Config) * len(p['cfgs']) == ctypes.sizeof(cfgs)
