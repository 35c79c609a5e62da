"""Every reference experiment config (config/**/*.yml, 93 of them, as tests/golden/make_config_fixture.py
extracted them): its state-representation flags, room and robots give a simaps_config the C ABI
accepts (its room within this build's limits), and
simaps_num_channels equals the config's own num_input_channels -- the channel count the reference's
policy networks are built for (policies.py:40, 93; networks.py:7)."""
import json
import os

import pytest

from simaps import _lib, batch, constants as K

ROWS = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'reference_configs.json')))


def test_fixture_covers_every_config():
    assert len(ROWS) == 93
    assert sum(r['use_predicted_intention'] for r in ROWS) == 12


@pytest.mark.parametrize('row', ROWS, ids=[r['config'] for r in ROWS])
def test_channel_count_matches_the_config(row):
    robots = sum(sum(d.values()) for d in row['robot_config'])
    assert 1 <= robots <= _lib.MAX_ROBOTS
    for layout in ('hwc', 'chw'):
        cfg = batch.make_config(row['flags'], row['room_width'], row['room_length'], layout)
        assert (cfg.H, cfg.W) == K.padded_room_shape(row['room_width'], row['room_length'])
        assert _lib.lib.simaps_num_channels(cfg, robots) == row['num_input_channels'], row['config']
        assert _lib.lib.simaps_rec_cache_bytes(cfg) > 0, _lib.lib.simaps_last_error()  # (the C ABI's config check)


def test_every_config_has_a_scene():
    """synthetic.reference_config_scene (the GPU test's inputs) builds for every config, with its
    robots, its flags, and descriptors the C structs take."""
    from simaps import synthetic
    for k, row in enumerate(ROWS):
        s = synthetic.reference_config_scene(row, k)
        assert [r['type'] for r in s['robots']] == [t for g in row['robot_config'] for t, c in g.items() for _ in range(c)]
        assert all(s['flags'][f] == v for f, v in row['flags'].items())
        agents = [(0, a) for a in range(len(s['robots']))]
        robots, envs, ag, paths = batch.pack_descriptors([s], agents)
        assert len(robots) == len(s['robots']) and s['occupancy'].shape == (len(agents), s['H'], s['W'])
