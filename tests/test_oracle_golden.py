"""CPU: the oracle (oracle/) reproduces the reference's outputs bit for bit.

The goldens were produced by running the reference's own code (tests/golden/make_goldens.py).
These tests pin the oracle; the GPU tests then check the HIP path against the oracle.
"""
import hashlib
import os

import numpy as np
import pytest

import goldens as G
import oracle as O
from simaps import constants as K


def test_trig_cosdg_sindg_bitwise():
    g = G.load('trig.npz')
    c = np.array([O.cosdg(a) for a in g['angle']])
    s = np.array([O.sindg(a) for a in g['angle']])
    assert np.array_equal(c.view(np.int64), g['cosdg'].view(np.int64))
    assert np.array_equal(s.view(np.int64), g['sindg'].view(np.int64))


# rotate.npz: the reference's scipy.ndimage.rotate on an FMA-dgemv host (round-1 builder);
# rotate_plain.npz: on a plain-dgemv host (numpy 1.26.4 / OpenBLAS 0.3.23, AVX-512 Xeon).
ROTATE_GOLDENS = [('rotate.npz', 'fma'), ('rotate_plain.npz', 'plain')]


@pytest.mark.parametrize('n', [96, 136])
@pytest.mark.parametrize('name,rounding', ROTATE_GOLDENS)
def test_rotate_index_maps(n, name, rounding):
    g = G.load(name)
    assert str(g['rounding']) == rounding
    for k, a in enumerate(g['angle']):
        i0, i1, v = O.rotate_index_map(n, float(a), rounding)
        m = np.where(v, i0 * n + i1, -1).astype(np.int32)
        assert m.shape == tuple(g['shape_%d' % n][k]), a
        assert hashlib.sha256(m.tobytes()).digest() == g['sha_%d' % n][k].tobytes(), a
    for q in range(6):
        i0, i1, v = O.rotate_index_map(n, float(g['angle'][q * 97]), rounding)
        assert np.array_equal(np.where(v, i0 * n + i1, -1), g['full_%d_%d' % (n, q)])


def test_rotate_fixtures_named_by_their_rounding():
    """Every rotate fixture records the host rounding that produced it, and its file name is the one
    make_goldens.write_rotate gives that rounding, so regenerating the goldens on either kind of host
    writes only its own file (the no-argument run on a plain host overwrote rotate.npz)."""
    import glob
    src = open(os.path.join(G.GOLDEN, 'make_goldens.py')).read()
    assert "np.savez_compressed(os.path.join(HERE, 'rotate.npz')" not in src  # only write_rotate writes it
    files = sorted(glob.glob(os.path.join(G.GOLDEN, 'rotate*.npz')))
    assert {os.path.basename(f) for f in files} == {n for n, _ in ROTATE_GOLDENS}
    for f in files:
        r = str(np.load(f)['rounding'])
        assert r in K.ROTATE_ROUNDINGS
        assert os.path.basename(f) == ('rotate.npz' if r == 'fma' else 'rotate_%s.npz' % r)


def test_rotate_roundings_differ_on_the_goldens():
    """The two hosts' goldens really differ (so each mode is pinned by its own host), and the
    other mode misses some of each host's angles: ~4-6 % of the random headings."""
    a, b = G.load('rotate.npz'), G.load('rotate_plain.npz')
    assert np.array_equal(a['angle'], b['angle'])
    for n in (96, 136):
        diff = (a['sha_%d' % n] != b['sha_%d' % n]).any(axis=1)
        assert 0.02 < diff[:1500].mean() < 0.1, diff[:1500].mean()


def test_scene_descriptors_record_their_rounding():
    """every committed scene descriptor carries the rotate rounding of the host
    whose reference run rendered it (make_goldens.py records K.host_rotate_rounding(), never
    synthetic.make_scene's default), so the loader needs no default and a regeneration with new
    seeds cannot produce fixtures whose label contradicts their content."""
    import glob
    import json
    n = 0
    for f in sorted(glob.glob(os.path.join(G.GOLDEN, 'scene_*.npz'))):
        z = np.load(f, allow_pickle=False)
        for k in z.files:
            if k.endswith('_scene'):
                assert json.loads(str(z[k])).get('rotate_rounding') in K.ROTATE_ROUNDINGS, (os.path.basename(f), k)
                n += 1
    assert n >= 27 + 14 + 4
    src = open(os.path.join(G.GOLDEN, 'make_goldens.py')).read()
    assert "dict(synthetic.make_scene(cfg, e), rotate_rounding=host)" in src


def test_host_rotate_rounding_is_a_known_form():
    assert K.host_rotate_rounding() in K.ROTATE_ROUNDINGS


def test_edt_feature_transform():
    g = G.load('edt.npz')
    for q in range(24):
        assert np.array_equal(O.edt_indices(g['in_%d' % q]), g['ft_%d' % q]), q


def test_bresenham_line():
    g = G.load('line.npz')
    off = g['off']
    for k, (r0, c0, r1, c1) in enumerate(g['ends']):
        rr, cc = O.line(int(r0), int(c0), int(r1), int(c1))
        assert np.array_equal(rr, g['rr'][off[k]:off[k + 1]]) and np.array_equal(cc, g['cc'][off[k]:off[k + 1]])


def test_linspace_ramp():
    g = G.load('linspace.npz')
    off = g['off']
    for k, (a, b, n) in enumerate(zip(g['start'], g['seg'], g['n'])):
        v = np.clip(O.linspace(1 - a, 1 - (a + b), int(n)), 0, 1)
        assert np.array_equal(v.view(np.int64), g['vals'][off[k]:off[k + 1]].view(np.int64))


def test_selems_and_grey_dilation():
    g = G.load('selem.npz')
    for r in range(9):
        assert np.array_equal(O.disk(r), g['disk_%d' % r])
    assert np.array_equal(O.grey_dilation_cross(g['grey_in']), g['grey_out'])


def test_robot_masks():
    g = G.load('masks.npz')
    for t in K.ROBOT_TYPES:
        assert np.array_equal(O.robot_mask(t), g[t])
    assert np.array_equal(O.robot_mask('lifting_robot', show_lifted_cube=True), g['lifting_robot_with_cube'])


def test_spfa_demo_known_answer():
    """shortest_paths/demo.py:33-52 sample: distance 136.46806, image, 12 more sources."""
    g = G.load('sssp.npz')
    img = O.spfa_image(g['demo_cspace'], (75, 156))
    assert np.array_equal(img.view(np.int32), g['demo_image'].view(np.int32))
    assert img[131, 112] == g['demo_distance']
    assert abs(float(g['demo_distance']) - 136.46806) < 1e-4
    assert (img >= 0).sum() == 5489
    for (i, j), sha in zip(g['demo_sources'], g['demo_sha']):
        im = O.spfa_image(g['demo_cspace'], (int(i), int(j)))
        assert hashlib.sha256(im.tobytes()).digest() == sha.tobytes()


def test_spfa_random_grids():
    g = G.load('sssp.npz')
    for q in range(10):
        im = O.spfa_image(g['rand_grid_%d' % q], tuple(int(x) for x in g['rand_src_%d' % q]))
        assert np.array_equal(im.view(np.int32), g['rand_img_%d' % q].view(np.int32)), q


CASES = list(G.scene_cases())


@pytest.mark.parametrize('case', CASES, ids=['%s-e%d-a%d' % c[:3] for c in CASES])
def test_agent_state_matches_reference(case):
    cfg, e, a, scene, pre, z = case
    ao = O.AgentOracle(scene, a)
    i0, j0, h, w = K.room_rect(scene['room_width'], scene['room_length'])
    assert np.array_equal(ao.cspace[i0:i0 + h, j0:j0 + w], z[pre + 'cspace_rect'])
    assert ao.cspace.sum() == z[pre + 'cspace_rect'].sum()
    assert np.array_equal(ao.closest, z[pre + 'closest'])
    srcs = []
    if scene['flags']['use_shortest_path_to_receptacle_map']:
        srcs.append(('receptacle', scene['receptacle_position']))
    if scene['flags']['use_shortest_path_map']:
        srcs.append(('robot', scene['robots'][a]['position']))
    for name, pos in srcs:
        ref = z[pre + 'src_%s' % name]
        assert O.position_to_pixel_indices(pos[0], pos[1], ao.shape) == (ref[0], ref[1])
        assert ao.snap(pos) == (ref[2], ref[3])
        img = O.spfa_image(ao.cspace, (ref[2], ref[3]))
        assert np.array_equal(img[i0:i0 + h, j0:j0 + w].view(np.int32), z[pre + 'sp_%s_rect' % name].view(np.int32))
    assert np.array_equal(ao.global_overhead_map(), z[pre + 'global_overhead'])
    assert np.array_equal(ao.global_robot_map(seg=False), z[pre + 'global_robot'])
    if scene['flags']['use_intention_map']:
        gi = ao.global_intention_map(scene['flags']['intention_map_encoding'])
        assert np.array_equal(gi.view(np.int32), z[pre + 'global_intention'].view(np.int32))
    if scene['flags']['use_history_map']:
        gh = ao.global_intention_map('history')
        assert np.array_equal(gh.view(np.int32), z[pre + 'global_history'].view(np.int32))
    st = ao.get_state()
    ref = z[pre + 'state']
    assert st.shape == ref.shape and st.dtype == np.float32
    assert np.array_equal(st.view(np.int32), ref.view(np.int32))


def test_oracle_shortest_path_distance_vs_reference():
    """Reward lookups: Mapper.distance_to_receptacle / OccupancyMap.
    shortest_path_distance (envs.py:2190-2194, 2507-2512) from the reference itself."""
    from simaps import synthetic
    z = G.load('sp_distance.npz')
    keys = sorted(k[:-len('_dist')] for k in z.files if k.endswith('_dist'))
    assert len(keys) >= 20
    for key in keys:
        cfg, rest = key.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        ao = O.AgentOracle(synthetic.make_scene(cfg, 40 + e), a)
        src = z[key + '_src']
        got = [ao.shortest_path_distance((src[0], src[1]), (x, y)) for x, y in z[key + '_queries']]
        assert got == list(z[key + '_dist']), key


def test_oracle_shortest_path_vs_reference():
    """Movement paths: OccupancyMap.shortest_path / GridGraph.shortest_path
    (envs.py:2478-2505, pyx:121-154) from the reference itself, exactly."""
    from simaps import synthetic
    z = G.load('paths.npz')
    keys = sorted(k[:-len('_path')] for k in z.files if k.endswith('_path') and not k.startswith('demo'))
    cache = {}
    for key in keys:
        head, q = key.rsplit('_q', 1)
        cfg, rest = head.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        if (cfg, e, a) not in cache:
            cache[(cfg, e, a)] = O.AgentOracle(synthetic.make_scene(cfg, 60 + e), a)
        got = np.array(cache[(cfg, e, a)].shortest_path(z[key + '_src'], z[key + '_tgt']), dtype=np.float64)
        assert np.array_equal(got, z[key + '_path']), key
    for q in range(3):
        got = np.array(O.grid_shortest_path(G.load('sssp.npz')['demo_cspace'], z['demo_%d_src' % q], z['demo_%d_tgt' % q]))
        assert np.array_equal(got.reshape(-1, 2), z['demo_%d_path' % q]), q


def test_oracle_ingest_vs_reference():
    """Observation ingest: Mapper.update with the reference's own
    Camera.capture_image on the committed depth / segmentation frames, exactly."""
    from simaps import camera, synthetic
    z = G.load('ingest.npz')
    for cfg, kind in (('lifting_4-small_divider', 'forward'), ('pushing_4-large_empty', 'overhead')):
        s = synthetic.make_scene(cfg, 80)
        for a in range(2):
            k = '%s_a%d' % (cfg, a)
            ov, oc = s['overhead'][a].copy(), s['occupancy'][a].copy()
            r = s['robots'][a]
            spec = camera.CAMERAS[kind]
            O.ingest(ov, oc, z[k + '_depth'], z[k + '_seg'].astype(np.int32),
                     spec.params(r['position'][0], r['position'][1], r['heading']), spec, synthetic.SEG_IDS,
                     s['receptacle_position'] is not None)
            assert np.array_equal(ov.view(np.int32), z[k + '_overhead'].view(np.int32)), k
            assert np.array_equal(oc, z[k + '_occupancy']), k


def test_oracle_grid_shortest_path_vs_reference():
    """GridGraph.shortest_path on raw cells (pyx:121-154): demo sample + multi-valued random grids."""
    z = G.load('grid_paths.npz')
    demo = G.load('sssp.npz')['demo_cspace']
    for k in sorted(k[:-4] for k in z.files if k.startswith('demo_') and k.endswith('_src')):
        got = np.array(O.grid_shortest_path(demo, z[k + '_src'], z[k + '_tgt'])).reshape(-1, 2)
        assert np.array_equal(got, z[k + '_path']), k
    for m in range(12):
        for k in range(6):
            key = 'rand_%d_%d' % (m, k)
            got = np.array(O.grid_shortest_path(z['rand_%d_grid' % m], z[key + '_src'], z[key + '_tgt'])).reshape(-1, 2)
            assert np.array_equal(got, z[key + '_path']), key


def test_oracle_maze_paths_vs_reference():
    """OccupancyMap.shortest_path on the maze environments (large_doors / tunnels / rooms) from the
    reference itself; the longest path bounds the intention path against SIMAPS_MAX_PATH."""
    from simaps import _lib, synthetic
    z = G.load('maze_paths.npz')
    assert int(z['longest_path']) + 1 <= _lib.MAX_PATH
    keys = sorted(k[:-len('_path')] for k in z.files if k.endswith('_path') and k != 'longest_path')
    cache = {}
    for key in keys:
        head, q = key.rsplit('_q', 1)
        cfg, rest = head.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        if (cfg, e, a) not in cache:
            cache[(cfg, e, a)] = O.AgentOracle(synthetic.make_scene(cfg, 70 + e, observe_all=True), a)
        got = np.array(cache[(cfg, e, a)].shortest_path(z[key + '_src'], z[key + '_tgt']), dtype=np.float64)
        assert np.array_equal(got, z[key + '_path']), key


@pytest.mark.parametrize('cfg', ['lifting_4-small_divider', 'pushing_4-large_empty'])
def test_rotate_rounding_changes_reference_states(cfg):
    """On the rounding-sensitive headings of scene_rot-plain_* the plain oracle reproduces the
    reference (test_agent_state_matches_reference) while the FMA form misses most stacks: the
    centre-pixel shift the round-2 verdict measured (sp channels by 1/96 x scale, intention up to
    0.9)."""
    cases = [c for c in CASES if c[5].zip.filename.endswith('scene_rot-plain_%s.npz' % cfg)]
    assert len(cases) == 8
    differ = 0
    for _, e, a, scene, pre, z in cases:
        got = O.AgentOracle(dict(scene, rotate_rounding='fma'), a).get_state()
        differ += not np.array_equal(got.view(np.int32), z[pre + 'state'].view(np.int32))
    assert differ >= 4, differ


def test_camera_params_batch_bitwise():
    """CameraSpec.params_batch (what StateBatch.prepare_ingest packs) equals the per-robot params()
    restatement of _get_camera_params (envs.py:1974-2008) bitwise, both cameras, including headings
    on exact multiples of pi / 2 and -0."""
    from simaps import camera
    rs = np.random.RandomState(11)
    poses = np.stack([rs.uniform(-3, 3, 4096), rs.uniform(-3, 3, 4096), rs.uniform(-7, 7, 4096)], 1)
    poses[:6, 2] = [0.0, -0.0, np.pi, -np.pi, np.pi / 2, -np.pi / 2]
    for kind, spec in camera.CAMERAS.items():
        want = np.array([spec.params(*p) for p in poses.tolist()], dtype=np.float64)
        got = spec.params_batch(poses)
        assert got.shape == (4096, 9) and np.array_equal(got.view(np.int64), want.view(np.int64)), kind
