"""GPU tests of get_state(save_figures=True) (envs.py:2115-2182): the whole-grid
maps simaps_global_maps exports are bit for bit the reference's own (the scene goldens' global_overhead /
global_robot / global_intention / global_history, written by make_goldens.py's run_agent from the
unmodified Mapper), and the PNGs VectorEnvObservations.get_state(save_figures=True) writes have the
pixels the reference's to_uint8_image / enlarge_image path gives for the oracle's maps."""
import numpy as np
import pytest
import torch

import goldens as G
import oracle as O

pytestmark = pytest.mark.gpu

CASES = list(G.scene_cases())


@pytest.fixture(scope='module')
def M():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a GPU (run with -m gpu on an MI355X)')
    from simaps import _lib, batch, figures, vector_env
    return _lib, batch, figures, vector_env


@pytest.mark.parametrize('case', range(len(CASES)))
def test_global_maps_vs_reference(M, case):
    _lib, batch, figures, vector_env = M
    cfg, e, a, scene, pre, z = CASES[case]
    b = batch.StateBatch([scene], agents=[(0, a)])
    g = {k: v[0].cpu().numpy() for k, v in b.global_maps().items()}
    _lib.check_faults()
    for name, key in (('overhead', 'global_overhead'), ('robot', 'global_robot'), ('intention', 'global_intention'),
                      ('history', 'global_history')):
        if pre + key not in z.files:
            continue
        if name == 'robot' and not scene['flags']['use_robot_map']:
            continue
        want = z[pre + key].astype(np.float32)
        assert name in g, name
        assert np.array_equal(g[name].view(np.int32), want.view(np.int32)), (cfg, name)


def _png_pixels(path):
    from PIL import Image
    return np.asarray(Image.open(path))


@pytest.mark.parametrize('cfg', ['lifting_4-small_divider', 'lifting_2_pushing_2-large_empty-all',
                                 'lifting_4-small_divider-history', 'lifting_4-large_empty-nonspatial'])
def test_save_figures_pngs_match_the_oracle(M, cfg, tmp_path):
    """Every PNG of get_state(save_figures=True) for every robot of two envs (one not awaiting, so no
    figures) against the same writer fed with the oracle's global maps and states."""
    _lib, batch, figures, vector_env = M
    from simaps import synthetic
    scenes = [synthetic.make_scene(cfg, 300 + e) for e in range(2)]
    obs = vector_env.VectorEnvObservations(scenes)
    awaiting = [[True] * len(s['robots']) for s in scenes]
    awaiting[1][0] = False
    st = obs.get_state(awaiting=awaiting, save_figures=True, numpy=True, figures_dir=str(tmp_path / 'gpu'))
    n = 0
    for e, s in enumerate(scenes):
        for a in range(len(s['robots'])):
            d = tmp_path / 'gpu' / ('robot_id_%d_%d' % (e, a))
            if not awaiting[e][a]:
                assert not d.exists()
                continue
            ao = O.AgentOracle(s, a)
            f = s['flags']
            gm = {'overhead': ao.global_overhead_map()}
            if f['use_robot_map']:
                gm['robot'] = ao.global_robot_map(seg=False)
            if f['use_shortest_path_to_receptacle_map']:
                gm['sp_receptacle'] = ao._sp_global(s['receptacle_position'])
            if f['use_shortest_path_map']:
                gm['sp_robot'] = ao._sp_global(s['robots'][a]['position'])
            if f['use_history_map']:
                gm['history'] = ao.global_intention_map('history')
            if f['use_intention_map']:
                gm['intention'] = ao.global_intention_map(f['intention_map_encoding'])
            ref_dir = tmp_path / 'oracle' / ('robot_id_%d_%d' % (e, a))
            want = figures.save_state_figures(ref_dir, f, s['room_length'], s['room_width'], len(s['robots']),
                                              O.agent_state(s, a), gm)
            got = sorted(p.name for p in d.iterdir())
            assert got == sorted(p.name for p in want)
            for p in want:
                assert np.array_equal(_png_pixels(d / p.name), _png_pixels(p)), (e, a, p.name)
                n += 1
            # the states returned are the rendered ones, unchanged by the figure path
            grp = [k for k, g in enumerate(obs.groups[e]) if a in g][0]
            assert np.array_equal(st[e][grp][obs.groups[e][grp].index(a)].view(np.int32),
                                  O.agent_state(s, a).view(np.int32))
    assert n >= 20


def test_save_figures_writes_the_occupancy_figure(M, tmp_path):
    """env.show_occupancy_maps (envs.py:2180-2182): the OccupancyMap passed for a figured robot saves its
    figure as global-occupancy-map.png next to the map PNGs; robots without one get none."""
    _lib, batch, figures, vector_env = M
    from simaps import synthetic
    s = synthetic.make_scene('lifting_4-small_divider', 410)
    obs = vector_env.VectorEnvObservations([s])
    om = vector_env.OccupancyMap(s['robots'][1]['type'], s['room_length'], s['room_width'], show_map=True)
    om.occupancy_map = s['occupancy'][1]
    om._update_map_visualization()
    obs.get_state(save_figures=True, numpy=True, figures_dir=str(tmp_path), occupancy_maps={(0, 1): om})
    om.save_figure(tmp_path / 'want.png')
    got = tmp_path / 'robot_id_0_1' / 'global-occupancy-map.png'
    assert np.array_equal(_png_pixels(got), _png_pixels(tmp_path / 'want.png'))
    assert not (tmp_path / 'robot_id_0_0' / 'global-occupancy-map.png').exists()
    assert (tmp_path / 'robot_id_0_0' / 'global-overhead-map.png').exists()
