"""GPU parity: the HIP path (through the C ABI) against the reference goldens and the oracle.

Bar (BASELINE.json north_star): bit-exact for the integer channels / intermediates (cspace,
snapped sources), and within 1e-5 for float channels -- we assert BIT-EXACT everywhere except
the nonspatial intention channels, whose fp64 sin/cos/atan2 come from the device libm (OCML)
instead of glibc and may differ in the last f32 bit (tolerance 1e-7 absolute there).
"""
import numpy as np
import pytest
import torch

import goldens as G
import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def S():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a GPU (run with -m gpu on an MI355X)')
    from simaps import batch, constants, synthetic
    return batch, constants, synthetic


def _bitwise(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(a.view(np.int32), b.view(np.int32))


def _nonspatial_slice(flags, nr):
    if not (flags['use_intention_channels'] and flags['intention_channel_encoding'] == 'nonspatial'):
        return None
    c0 = 1 + sum(bool(flags[k]) for k in ('use_robot_map', 'use_distance_to_receptacle_map',
                                          'use_shortest_path_to_receptacle_map', 'use_shortest_path_map',
                                          'use_history_map', 'use_intention_map'))
    return slice(c0, c0 + 2 * (nr - 1))


def _check_state(got, ref, flags, nr):
    ns = _nonspatial_slice(flags, nr)
    if ns is None:
        assert _bitwise(got, ref), 'max abs diff %g' % np.abs(got - ref).max()
    else:
        mask = np.ones(got.shape[-1], bool)
        mask[ns] = False
        assert _bitwise(np.ascontiguousarray(got[..., mask]), np.ascontiguousarray(ref[..., mask]))
        assert np.abs(got[..., ns] - ref[..., ns]).max() <= 1e-7


GOLD = list(G.scene_cases())


@pytest.mark.parametrize('case', GOLD, ids=['%s-e%d-a%d' % c[:3] for c in GOLD])
def test_golden_scene_state_and_intermediates(S, case):
    batch, K, synthetic = S
    cfg, e, a, scene, pre, z = case
    b = batch.StateBatch([scene], agents=[(0, a)], layout='hwc' if e == 0 else 'chw')
    dbg = b.alloc_debug()
    st = b.as_hwc(b.render(debug=dbg))
    torch.cuda.synchronize()
    flags = scene['flags']
    assert int(dbg['status'][0]) & 0xff == 0
    assert np.array_equal(dbg['cspace'][0].cpu().numpy(), z[pre + 'cspace_rect'])
    src = dbg['sources'][0].cpu().numpy()
    dist = dbg['dist'][0].cpu().numpy()
    if flags['use_shortest_path_to_receptacle_map']:
        assert np.array_equal(src[0], z[pre + 'src_receptacle'])
        assert _bitwise(dist[0], z[pre + 'sp_receptacle_rect'])
    if flags['use_shortest_path_map']:
        assert np.array_equal(src[1], z[pre + 'src_robot'])
        assert _bitwise(dist[1], z[pre + 'sp_robot_rect'])
    _check_state(st[0].cpu().numpy(), z[pre + 'state'], flags, len(scene['robots']))


def test_layout_chw_matches_hwc(S):
    batch, K, synthetic = S
    scenes = [synthetic.make_scene('lifting_2_pushing_2-large_empty-all', e) for e in range(3)]
    hwc = batch.StateBatch(scenes, layout='hwc').render().cpu().numpy()
    chw = batch.StateBatch(scenes, layout='chw').render().cpu().numpy()
    assert _bitwise(np.transpose(chw, (0, 2, 3, 1)), hwc)


@pytest.mark.parametrize('cfg', ['lifting_1-small_empty', 'lifting_4-small_divider', 'pushing_4-large_empty',
                                 'lifting_2_throwing_2-large_empty', 'rescue_4-small_empty',
                                 'lifting_4-small_divider-history', 'lifting_4-large_empty-line',
                                 'lifting_4-small_empty-circle', 'lifting_4-small_divider-spatial',
                                 'lifting_4-large_empty-nonspatial', 'lifting_2_pushing_2-large_empty-all',
                                 'lifting_4-large_doors', 'lifting_4-large_tunnels', 'lifting_4-large_rooms',
                                 'lifting_2_throwing_2-large_doors', 'lifting_4-large_rooms-history'])
@pytest.mark.parametrize('rounding', ['fma', 'plain'])
def test_oracle_parity_fresh_seeds(S, cfg, rounding):
    """Seeds never used for the goldens: every agent of 6 envs vs the (golden-pinned) oracle, in
    both host roundings of scipy.ndimage.rotate's out_center (rotate.npz / rotate_plain.npz)."""
    batch, K, synthetic = S
    scenes = [dict(synthetic.make_scene(cfg, 100 + e), rotate_rounding=rounding) for e in range(6)]
    b = batch.StateBatch(scenes)
    st = b.as_hwc(b.render()).cpu().numpy()
    for n, (e, a) in enumerate(b.agents):
        _check_state(st[n], O.agent_state(scenes[e], a), scenes[e]['flags'], len(scenes[e]['robots']))


@pytest.mark.parametrize('scale', [-0.5, 0.0, 3.0])
def test_shortest_path_map_scale_signs(S, scale):
    """The distance phase scales with |scale| and flips signs afterwards; unreachable / blocked
    cells become the scaled max (envs.py:2288-2300) and cval pixels stay +0, for any scale."""
    batch, K, synthetic = S
    for cfg in ['lifting_4-small_divider', 'lifting_2_pushing_2-large_empty-all', 'rescue_4-small_empty']:
        scenes = [synthetic.make_scene(cfg, 200 + e) for e in range(2)]
        for sc in scenes:
            sc['flags'] = dict(sc['flags'], shortest_path_map_scale=scale)
        b = batch.StateBatch(scenes)
        st = b.as_hwc(b.render()).cpu().numpy()
        for n, (e, a) in enumerate(b.agents):
            _check_state(st[n], O.agent_state(scenes[e], a), scenes[e]['flags'], len(scenes[e]['robots']))


def test_full_size_lifting_4_small_divider_properties(S):
    """BASELINE configs[1] size (64 envs x 4 agents): determinism, channel invariants, and a
    seeded sample of agents against the oracle."""
    batch, K, synthetic = S
    scenes = [synthetic.make_scene('lifting_4-small_divider', e) for e in range(64)]
    b = batch.StateBatch(scenes)
    s1 = b.as_hwc(b.render()).cpu().numpy()
    s2 = b.as_hwc(b.render()).cpu().numpy()
    assert _bitwise(s1, s2)                       # idempotent / deterministic
    assert s1.shape == (256, 96, 96, 5)
    assert np.all(s1[..., 0] <= 1) and np.all(s1 >= 0)
    assert np.all(s1[..., 2].reshape(256, -1).min(1) == 0) and np.all(s1[..., 3].reshape(256, -1).min(1) == 0)
    assert set(np.unique(s1[..., 1])) <= {0.0, 0.5, 1.0}
    assert set(np.unique(s1[..., 0])) <= {k / 8 for k in range(9)}
    rs = np.random.RandomState(7)
    for n in rs.choice(256, 12, replace=False):
        e, a = b.agents[n]
        assert _bitwise(s1[n], O.agent_state(scenes[e], a))


def _channel_invariants(st, flags):
    """Size-independent properties of rendered stacks (N, 96, 96, C), by channel (envs.py:2071-2113)."""
    N = st.shape[0]
    assert np.all(np.isfinite(st))
    c = 0
    assert set(np.unique(st[..., c])) <= {k / 8 for k in range(9)}      # overhead: seg codes k / 8
    c += 1
    if flags['use_robot_map']:
        assert set(np.unique(st[..., c])) <= {0.0, 0.5, 1.0}
        c += 1
    if flags['use_distance_to_receptacle_map']:
        c += 1
    for k in ('use_shortest_path_to_receptacle_map', 'use_shortest_path_map'):
        if flags[k]:                                                     # local min-subtract (envs.py:2213-2216)
            assert np.all(st[..., c].reshape(N, -1).min(1) == 0)
            c += 1
    if flags['use_history_map'] or flags['use_intention_map']:
        assert np.all(st[..., c] >= 0) and np.all(st[..., c] <= max(1.0, flags['intention_map_scale']))


@pytest.mark.parametrize('cfg,envs', [('pushing_4-large_empty', 256), ('lifting_2_throwing_2-large_empty', 1024),
                                      ('rescue_4-small_empty', 2048), ('lifting_4-large_tunnels', 256),
                                      ('lifting_4-large_rooms', 256)])
def test_full_size_baseline_configs(S, cfg, envs):
    """The other BASELINE configs at their full single-launch sizes (1,024 / 4,096 / 8,192 stacks,
    i.e. 4-32 workgroups per CU back to back): no device fault, status clean for every agent,
    deterministic, channel invariants, and a seeded sample of agents bitwise against the oracle."""
    from simaps import _lib
    batch, K, synthetic = S
    scenes = [synthetic.make_scene(cfg, 3000 + e) for e in range(envs)]
    b = batch.StateBatch(scenes)
    status = torch.full((b.N,), -1, dtype=torch.int32, device=b.device)
    s1 = b.as_hwc(b.render(debug={'status': status})).cpu().numpy()
    _lib.check_faults()
    st = status.cpu().numpy()
    assert np.all(st & 0xff == 0), 'status bits set for %d agents' % int((st & 0xff != 0).sum())
    assert np.all(st >> 8 > 0)                                           # every agent's SSSP converged
    s2 = b.as_hwc(b.render()).cpu().numpy()
    assert _bitwise(s1, s2)
    _channel_invariants(s1, scenes[0]['flags'])
    rs = np.random.RandomState(11)
    for n in sorted(rs.choice(b.N, 46, replace=False)) + [0, b.N - 1]:
        e, a = b.agents[n]
        assert _bitwise(s1[n], O.agent_state(scenes[e], a)), (cfg, n)


def test_snap_slow_path_and_idle(S):
    """Agents pressed against walls / divider (query pixel not free -> EDT snap), all robots idle."""
    batch, K, synthetic = S
    scenes = []
    for e in range(8):
        s = synthetic.make_scene('lifting_4-small_divider', 300 + e, observe_all=True)
        for k, r in enumerate(s['robots']):
            x = (-0.5 + 0.03) if k % 2 == 0 else (0.5 - 0.02 - 0.01 * e)
            y = (0.25 - 0.02) if k < 2 else (-0.25 + 0.04)
            r['position'] = (x, y, 0)
            r['waypoint_positions'][0] = r['position']
            r['idle'] = e % 2 == 0
        scenes.append(s)
    b = batch.StateBatch(scenes)
    dbg = b.alloc_debug()
    st = b.as_hwc(b.render(debug=dbg)).cpu().numpy()
    src = dbg['sources'].cpu().numpy()
    assert (src[:, 1, :2] != src[:, 1, 2:]).any(), 'expected at least one snapped robot source'
    for n, (e, a) in enumerate(b.agents):
        assert _bitwise(st[n], O.agent_state(scenes[e], a))


def test_snap_ties_on_maze_walls(S):
    """EDT snap (scipy feature transform at the query, envs.py:2523-2524) for robots standing on the
    large_rooms / large_tunnels dividers: every robot source needs the slow path, many with
    equidistant free cells (the lowest minimal column wins, like scipy's envelope scan)."""
    batch, K, synthetic = S
    rs = np.random.RandomState(17)
    scenes = []
    for e in range(24):
        cfg = 'lifting_4-large_rooms' if e % 2 == 0 else 'lifting_4-large_tunnels'
        s = synthetic.make_scene(cfg, 900 + e, observe_all=e % 3 == 0)
        for k, r in enumerate(s['robots']):
            if cfg.endswith('rooms'):  # on the cross walls (through the room centre), +- a few pixels
                x, y = (rs.uniform(-0.3, 0.3), rs.randint(-3, 4) / 96.0) if k % 2 else (rs.randint(-3, 4) / 96.0, rs.uniform(-0.3, 0.3))
            else:  # inside the tunnel walls
                x, y = rs.uniform(-0.45, 0.45), rs.uniform(-0.1, 0.1)
            r['position'] = (float(x), float(y), 0)
            r['waypoint_positions'][0] = r['position']
        scenes.append(s)
    b = batch.StateBatch(scenes)
    dbg = b.alloc_debug()
    st = b.as_hwc(b.render(debug=dbg)).cpu().numpy()
    src = dbg['sources'].cpu().numpy()
    snapped = int((src[:, 1, :2] != src[:, 1, 2:]).any(axis=1).sum())
    assert snapped >= 48, snapped
    for n, (e, a) in enumerate(b.agents):
        assert _bitwise(st[n], O.agent_state(scenes[e], a)), (n, e, a)


def test_edge_poses_and_degenerate_paths(S):
    """The fp64 index rules at their edges: headings on exact multiples of 45 deg (and +-pi, +-0,
    whole degrees), positions on pixel boundaries (position_to_pixel_indices floors exactly there,
    envs.py:2391-2397), zero-length path segments and a waypoint index at the end of the path."""
    batch, K, synthetic = S
    rs = np.random.RandomState(23)
    heads = [k * np.pi / 4 for k in range(-4, 5)] + [-0.0, np.radians(30.0), np.radians(-135.0), np.radians(1.0),
                                                     1e-12, -1e-12, np.nextafter(np.pi, 0.0)]
    k = 0
    for c, cfg in enumerate(['lifting_4-small_divider', 'rescue_4-small_empty', 'lifting_4-large_empty-line',
                             'lifting_2_pushing_2-large_empty-all']):
        scenes = [synthetic.make_scene(cfg, 700 + 2 * c + e) for e in range(2)]
        for s in scenes:
            H, W = s['H'], s['W']
            for r in s['robots']:
                j, i = rs.randint(W // 2 - 30, W // 2 + 30), rs.randint(H // 2 - 15, H // 2 + 15)
                x, y = (j - W / 2) / 96.0, (H / 2 - i) / 96.0   # on a pixel corner
                if k % 3 == 1:
                    x = np.nextafter(x, -1.0)                     # just below it
                r['position'] = (float(x), float(y), 0)
                r['heading'] = float(heads[k % len(heads)])
                r['idle'] = False
                wps = [r['position']] * 2 + list(r['waypoint_positions'][1:])
                r['waypoint_positions'] = wps
                r['waypoint_index'] = len(wps) - 1 if k % 2 else 1
                k += 1
        b = batch.StateBatch(scenes)
        st = b.as_hwc(b.render()).cpu().numpy()
        for n, (e, a) in enumerate(b.agents):
            _check_state(st[n], O.agent_state(scenes[e], a), scenes[e]['flags'], len(scenes[e]['robots']))


def test_sssp_grid_demo_known_answer(S):
    """shortest_paths/demo.py sample: distance 136.46806 and the full image, + 12 more sources."""
    batch, K, synthetic = S
    g = G.load('sssp.npz')
    grid = g['demo_cspace']
    fr = np.argwhere(grid > 0)
    (i0, j0), (i1, j1) = fr.min(0), fr.max(0)
    win = (int(i0), int(j0), int(i1 - i0 + 1), int(j1 - j0 + 1))
    srcs = [(75, 156)] + [tuple(int(x) for x in p) for p in g['demo_sources']]
    grids = torch.from_numpy(np.repeat(grid[None], len(srcs), 0)).cuda()
    out = batch.sssp_grid(grids, torch.tensor(srcs, dtype=torch.int32), window=win).cpu().numpy()
    assert _bitwise(out[0], g['demo_image'])
    assert out[0][131, 112] == g['demo_distance']
    for q, (i, j) in enumerate(srcs[1:]):
        assert _bitwise(out[q + 1], O.spfa_image(grid, (i, j)))


def test_sssp_grid_random(S):
    batch, K, synthetic = S
    g = G.load('sssp.npz')
    for q in range(10):
        grid = g['rand_grid_%d' % q]
        src = torch.tensor([tuple(int(x) for x in g['rand_src_%d' % q])], dtype=torch.int32)
        out = batch.sssp_grid(torch.from_numpy(grid[None].copy()).cuda(), src).cpu().numpy()
        assert _bitwise(out[0], g['rand_img_%d' % q]), q


def _room_grids(n, h, w, seed):
    """n uint8 grids [h + 4, w + 4] whose free cells lie in the window (2, 2, h, w): a divider wall
    with one gap (long detours) and random blocks; one random free source cell each."""
    rs = np.random.RandomState(seed)
    grids, srcs = [], []
    for _ in range(n):
        g = np.zeros((h + 4, w + 4), np.uint8)
        g[2:2 + h, 2:2 + w] = 1
        c = 2 + w // 2 + rs.randint(-8, 9)
        g[2:2 + h, c] = 0
        gap = 2 + rs.randint(0, h - 6)
        g[gap:gap + 5, c] = 1
        for _ in range(12):
            i, j = 2 + rs.randint(0, h - 4), 2 + rs.randint(0, w - 4)
            g[i:i + rs.randint(1, 5), j:j + rs.randint(1, 5)] = 0
        fr = np.argwhere(g > 0)
        grids.append(g)
        srcs.append(tuple(int(x) for x in fr[rs.randint(len(fr))]))
    return np.stack(grids), srcs


@pytest.mark.parametrize('h', [44, 92])
def test_sssp_grid_room_width_92(S, h):
    """Rooms 92 cells wide (the BASELINE rooms' pitch 95: the sweeps' compile-time asm loops, and the
    split-sweep variant when built with SIMAPS_SSSP_SPLIT_L / _S), with a divider: bitwise the SPFA."""
    batch, K, synthetic = S
    grids, srcs = _room_grids(6, h, 92, 40 + h)
    out = batch.sssp_grid(torch.from_numpy(grids).cuda(), torch.tensor(srcs, dtype=torch.int32),
                          window=(2, 2, h, 92)).cpu().numpy()
    for q in range(len(srcs)):
        assert _bitwise(out[q], O.spfa_image(grids[q], srcs[q])), q


@pytest.mark.parametrize('mode', ['random', 'eighths_and_negzero'])
def test_overhead_values_outside_seg_codes(S, mode):
    """Overhead maps holding values other than the SEG_VALUES codes k/8 (random floats, -0.0, a code
    the scene's seg values never use): the overhead channel gathers them unchanged, bit for bit."""
    batch, K, synthetic = S
    rs = np.random.RandomState(11)
    scenes = [synthetic.make_scene('lifting_4-small_divider', 900 + e) for e in range(4)]
    for e, s in enumerate(scenes):
        ov = s['overhead']
        if e % 2 == 0:   # envs 0, 2: perturbed; envs 1, 3 stay on the code path
            if mode == 'random':
                ov[:, 60:120, 60:160] = rs.rand(ov.shape[0], 60, 100).astype(np.float32)
            else:
                ov[:, 70:110, 70:150] = np.float32(7 / 8)    # a code no seg value of this scene uses
                ov[:, 90, 100] = np.float32(-0.0)             # -0.0 is not the code 0
                ov[:, 95, 101] = np.float32(0.3)              # not a multiple of 1/8
    b = batch.StateBatch(scenes)
    st = b.as_hwc(b.render()).cpu().numpy()
    for n, (e, a) in enumerate(b.agents):
        assert _bitwise(st[n], O.agent_state(scenes[e], a))
