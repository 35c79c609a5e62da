"""GPU tests of the drop-in host interface (simaps.vector_env) against the oracle.

VectorEnv.get_state structure (envs.py:322-323): list over robot groups of lists over robots,
None for robots not awaiting an action; GridGraph.shortest_path_image / _distance
(shortest_paths.pyx:156-167) including the per-source cache and a blocked source.
"""
import numpy as np
import pytest
import torch

import goldens as G
import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def V():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a GPU (run with -m gpu on an MI355X)')
    from simaps import synthetic, vector_env
    return synthetic, vector_env


def _key_epochs(b):
    """The launch epochs (top byte) present in a StateBatch's ingest key map."""
    return set(int(x) for x in np.unique(b._keys.cpu().numpy().view(np.uint64) >> np.uint64(56)))


def _bitwise(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(a.view(np.int32), b.view(np.int32))


@pytest.mark.parametrize('layout', ['hwc', 'chw'])
def test_get_state_structure_and_awaiting_subset(V, layout):
    synthetic, vector_env = V
    cfg = 'lifting_2_throwing_2-large_empty'       # two robot groups
    scenes = [synthetic.make_scene(cfg, 500 + e) for e in range(3)]
    obs = vector_env.VectorEnvObservations(scenes, layout=layout)
    rs = np.random.RandomState(3)
    awaiting = [[bool(rs.randint(2)) for _ in s['robots']] for s in scenes]
    awaiting[0] = [False] * 4                        # an env with nobody awaiting
    st = obs.get_state(awaiting=awaiting, numpy=True)
    full = obs.get_state(all_robots=True)
    assert len(st) == 3
    for e, s in enumerate(scenes):
        groups = vector_env.robot_groups(s)
        assert [len(g) for g in st[e]] == [len(g) for g in groups] == [2, 2]
        for g, idx in zip(st[e], groups):
            for x, a in zip(g, idx):
                if not awaiting[e][a]:
                    assert x is None
                    continue
                assert isinstance(x, np.ndarray) and x.shape == (96, 96, 5) and x.dtype == np.float32
                assert _bitwise(x, O.agent_state(s, a))
        for g, idx in zip(full[e], groups):
            for x, a in zip(g, idx):
                assert isinstance(x, torch.Tensor) and tuple(x.shape) == (96, 96, 5)
                assert _bitwise(x.cpu().numpy(), O.agent_state(s, a))


@pytest.mark.parametrize('layout', ['hwc', 'chw'])
def test_reuse_outputs_rings(V, layout):
    """reuse_outputs=2: the all-robots get_state renders into a ring of two device batches (views
    built once), and with numpy=True into a ring of pinned host copies; every call's states equal
    the oracle's bitwise, the same slot's views come back every second call (overwritten in
    place), and the awaiting-subset path is unaffected."""
    synthetic, vector_env = V
    cfg = 'lifting_2_throwing_2-large_empty'
    scenes = [synthetic.make_scene(cfg, 520 + e) for e in range(3)]
    want = {(e, a): O.agent_state(s, a) for e, s in enumerate(scenes) for a in range(len(s['robots']))}
    obs = vector_env.VectorEnvObservations(scenes, layout=layout, reuse_outputs=2)
    seen_dev, seen_host = [], []
    for call in range(4):
        dev = obs.get_state()
        host = obs.get_state(numpy=True)
        torch.cuda.synchronize()
        for e, s in enumerate(scenes):
            for gd, gh, idx in zip(dev[e], host[e], vector_env.robot_groups(s)):
                for xd, xh, a in zip(gd, gh, idx):
                    assert isinstance(xd, torch.Tensor) and isinstance(xh, np.ndarray)
                    assert xh.shape == (96, 96, 5) and xh.dtype == np.float32
                    assert _bitwise(xd.cpu().numpy(), want[(e, a)]) and _bitwise(xh, want[(e, a)]), (call, e, a)
        seen_dev.append(dev[0][0][0].data_ptr())
        seen_host.append(host[0][0][0].__array_interface__['data'][0])
    assert seen_dev[0] == seen_dev[2] != seen_dev[1] == seen_dev[3]
    assert seen_host[0] == seen_host[2] != seen_host[1] == seen_host[3]
    awaiting = [[a % 2 == 0 for a in range(len(s['robots']))] for s in scenes]
    sub = obs.get_state(awaiting=awaiting, numpy=True)
    for e, s in enumerate(scenes):
        for g, idx in zip(sub[e], vector_env.robot_groups(s)):
            for x, a in zip(g, idx):
                assert (x is None) == (not awaiting[e][a]) and (x is None or _bitwise(x, want[(e, a)]))


def test_get_state_nobody_awaiting(V):
    """A step where no robot awaits an action: every entry None, nothing launched, and the next
    step renders normally."""
    synthetic, vector_env = V
    scenes = [synthetic.make_scene('lifting_4-small_divider', 510 + e) for e in range(2)]
    obs = vector_env.VectorEnvObservations(scenes)
    st = obs.get_state(awaiting=[[False] * 4, [False] * 4], numpy=True)
    assert [[x is None for g in env for x in g] for env in st] == [[True] * 4, [True] * 4]
    st = obs.get_state(awaiting=[[False, True, False, False], [False] * 4], numpy=True)
    assert st[1][0] == [None] * 4 and _bitwise(st[0][0][1], O.agent_state(scenes[0], 1))


def test_update_descriptors_and_maps(V):
    synthetic, vector_env = V
    cfg = 'lifting_4-small_divider'
    a = [synthetic.make_scene(cfg, 600 + e) for e in range(2)]
    b = [synthetic.make_scene(cfg, 700 + e) for e in range(2)]
    obs = vector_env.VectorEnvObservations(a)
    obs.get_state()
    # new step: descriptors of b, maps of b for agent slots 1 and 6 only -> those two match the
    # oracle on a scene mixing b's descriptor with their own b maps
    occ = np.stack([b[e]['occupancy'][r] for e, r in [(0, 1), (1, 2)]])
    ovh = np.stack([b[e]['overhead'][r] for e, r in [(0, 1), (1, 2)]])
    obs.update(scenes=b, occupancy=occ, overhead=ovh, slots=[1, 6])
    st = obs.get_state(numpy=True)
    assert _bitwise(st[0][0][1], O.agent_state(b[0], 1))
    assert _bitwise(st[1][0][2], O.agent_state(b[1], 2))
    mixed = dict(b[0], occupancy=a[0]['occupancy'], overhead=a[0]['overhead'])
    assert _bitwise(st[0][0][0], O.agent_state(mixed, 0))   # slot 0 kept a's maps
    with pytest.raises(ValueError):
        obs.update(scenes=b[:1])


def test_gridgraph_dropin(V):
    synthetic, vector_env = V
    g = G.load('sssp.npz')
    grid = g['demo_cspace']
    gg = vector_env.GridGraph(grid)
    img = gg.shortest_path_image((75, 156))
    assert _bitwise(img, g['demo_image'])
    assert gg.shortest_path_distance((75, 156), (131, 112)) == float(g['demo_distance'])
    assert (75, 156) in gg._cache                     # _spfa_with_cache semantics
    # a blocked source: distance 0 at the source, -1 everywhere else (pyx:84-85, 110-112)
    blocked = tuple(int(x) for x in np.argwhere(grid == 0)[len(np.argwhere(grid == 0)) // 2])
    bi = gg.shortest_path_image(blocked)
    assert _bitwise(bi, O.spfa_image(grid, blocked))
    with pytest.raises(IndexError):
        gg.shortest_path_distance((75, 156), (10_000, 0))


def test_sp_distance_reference_goldens(V):
    """Reward lookups through simaps_sp_distance vs values produced by the
    reference's own Mapper.distance_to_receptacle / OccupancyMap.shortest_path_distance."""
    synthetic, vector_env = V
    from simaps import batch
    z = G.load('sp_distance.npz')
    keys = sorted(k[:-len('_dist')] for k in z.files if k.endswith('_dist'))
    by_cfg = {}
    for key in keys:
        cfg, rest = key.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        by_cfg.setdefault(cfg, []).append((e, a, key))
    for cfg, items in by_cfg.items():
        scenes = [synthetic.make_scene(cfg, 40 + e) for e in range(2)]
        b = batch.StateBatch(scenes)
        slots = [b.agents.index((e, a)) for e, a, _ in items]
        src = np.stack([z[k + '_src'] for _, _, k in items])
        tgt = np.stack([z[k + '_queries'] for _, _, k in items])
        got = b.shortest_path_distances(src, tgt, slots=slots).cpu().numpy()
        want = np.stack([z[k + '_dist'] for _, _, k in items])
        assert np.array_equal(got, want), cfg


def test_sp_distance_many_targets_vs_oracle(V):
    """130 targets per agent (three chunks of the kernel's lane-parallel fast snap), a third of them
    in walls / the divider / outside the room (the EDT slow path), some robots standing in walls."""
    synthetic, vector_env = V
    from simaps import batch
    scenes = [synthetic.make_scene('lifting_4-small_divider', 80 + e) for e in range(3)]
    rs = np.random.RandomState(9)
    for s in scenes:
        s['robots'][0]['position'] = (0.0, rs.uniform(-0.2, 0.2), 0)   # on the divider
    b = batch.StateBatch(scenes)
    Q = 130
    src = np.array([scenes[e]['robots'][a]['position'][:2] for e, a in b.agents])
    tgt = np.stack([rs.uniform(-0.3, 0.3, (b.N, Q)), rs.uniform(-0.3, 0.3, (b.N, Q))], -1)
    tgt[:, ::3, 0] = rs.choice([0.0, -0.5, 0.5, 0.55], (b.N, len(range(0, Q, 3))))  # divider, walls, outside
    got = b.shortest_path_distances(src, tgt).cpu().numpy()
    for n, (e, a) in enumerate(b.agents):
        ao = O.AgentOracle(scenes[e], a)
        assert got[n].tolist() == [ao.shortest_path_distance(src[n], t) for t in tgt[n]], (e, a)


def _sp_golden_items(z):
    keys = sorted(k[:-len('_dist')] for k in z.files if k.endswith('_dist'))
    by_cfg = {}
    for key in keys:
        cfg, rest = key.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        by_cfg.setdefault(cfg, []).append((e, a, key))
    return by_cfg


def test_receptacle_lookups_from_the_render_cache_reference_goldens(V):
    """Mapper.distance_to_receptacle answered from the receptacle arrays get_state
    left in the cache (the reference's GridGraph cache, shortest_paths.pyx:116-119, 156-163) -- after
    one render every lookup is a cache hit (simaps_sp_lookup, no SSSP) -- equals the reference's own
    values; so does the cold path (full SSSP, which then fills the cache) and the second, cached call."""
    synthetic, vector_env = V
    from simaps import batch
    z = G.load('sp_distance.npz')
    for cfg, items in _sp_golden_items(z).items():
        scenes = [synthetic.make_scene(cfg, 40 + e) for e in range(2)]
        if scenes[0]['receptacle_position'] is None:
            continue
        slots = None
        want = None
        for mode in ('render', 'cold'):
            b = batch.StateBatch(scenes)
            slots = [b.agents.index((e, a)) for e, a, _ in items]
            tgt = np.stack([z[k + '_queries'] for _, _, k in items])
            want = np.stack([z[k + '_dist'] for _, _, k in items])
            b.enable_receptacle_cache()
            if mode == 'render':
                b.render()
                assert (b._rec_ver == b._map_ver).all()           # every slot cached
            else:
                assert not (b._rec_ver[slots] == b._map_ver[slots]).any()
            got = b.receptacle_distances(tgt, slots=slots).cpu().numpy()
            assert np.array_equal(got, want), (cfg, mode)
            assert (b._rec_ver[slots] == b._map_ver[slots]).all()  # (the cold call filled the cache)
            again = b.receptacle_distances(tgt, slots=slots).cpu().numpy()
            assert np.array_equal(again, want), (cfg, mode, 'cached')


def test_receptacle_cache_follows_map_updates(V):
    """An ingest (and a set_maps) between the render and the lookups invalidates exactly those slots'
    cached arrays: their lookups run the SSSP on the new maps, the others stay cache hits, and all of
    them equal the oracle on the current maps -- also for blocked / outside targets (the EDT slow path
    rebuilt from the cached array) and in a batch whose render does not fill the cache (no
    shortest-path-to-receptacle channel: every first lookup is a miss)."""
    synthetic, vector_env = V
    from simaps import batch, camera
    spec = camera.CAMERAS['forward']
    rs = np.random.RandomState(21)
    for no_channel in (False, True):
        scenes = [synthetic.make_scene('lifting_4-small_divider', 660 + e) for e in range(3)]
        if no_channel:
            for sc in scenes:
                sc['flags'] = dict(sc['flags'], use_shortest_path_to_receptacle_map=False)
        b = batch.StateBatch(scenes)
        b.enable_receptacle_cache()
        b.render()
        Q = 70
        tgt = np.stack([rs.uniform(-0.3, 0.3, (b.N, Q)), rs.uniform(-0.3, 0.3, (b.N, Q))], -1)
        tgt[:, ::4, 0] = rs.choice([0.0, -0.5, 0.5, 0.55], (b.N, len(range(0, Q, 4))))  # divider, walls, outside

        def check(tag):
            got = b.receptacle_distances(tgt).cpu().numpy()
            for n, (e, a) in enumerate(b.agents):
                ao = O.AgentOracle(scenes[e], a)
                rec = scenes[e]['receptacle_position']
                assert got[n].tolist() == [ao.shortest_path_distance(rec, t) for t in tgt[n]], (tag, e, a)
        if not no_channel:
            assert (b._rec_ver == b._map_ver).all()
        check('after render')
        moved = [0, 5, 9]
        f = [synthetic.camera_images(scenes[e], a, 'forward', seed=31 + k) for k, (e, a) in
             enumerate(b.agents[k] for k in moved)]
        b.ingest(np.stack([x[0] for x in f]), np.stack([x[1] for x in f]).astype(np.int32), slots=moved)
        for k, (x, n) in enumerate(zip(f, moved)):
            e, a = b.agents[n]
            r = scenes[e]['robots'][a]
            O.ingest(scenes[e]['overhead'][a], scenes[e]['occupancy'][a], x[0], x[1],
                     spec.params(r['position'][0], r['position'][1], r['heading']), spec, synthetic.SEG_IDS,
                     scenes[e]['receptacle_position'] is not None)
        stale = b._rec_ver != b._map_ver
        assert sorted(np.nonzero(stale)[0].tolist()) == moved
        check('after ingest')
        occ = scenes[1]['occupancy'][2].copy()
        occ[60:70, 100:110] = 1   # a new obstacle in slot 6's map
        scenes[1]['occupancy'][2] = occ
        b.set_maps(occupancy=occ[None], slots=[6])
        assert (b._rec_ver != b._map_ver).sum() == 1
        check('after set_maps')


def _rec_check(b, scenes, tgt, tag, **kw):
    got = b.receptacle_distances(tgt, **kw).cpu().numpy()
    for n, (e, a) in enumerate(b.agents):
        ao = O.AgentOracle(scenes[e], a)
        rec = scenes[e]['receptacle_position']
        assert got[n].tolist() == [ao.shortest_path_distance(rec, t) for t in tgt[n]], (tag, e, a)


def test_receptacle_cache_after_graph_replayed_ingest(V):
    """an ingest captured into a graph changes the maps on every replay without a
    host-side version bump.  A render between the capture and a replay must not make the cache serve
    the pre-replay arrays: slots a captured ingest writes are never cache hits, and the lookups after
    the replay equal the oracle on the replayed maps."""
    synthetic, vector_env = V
    from simaps import batch, camera
    spec = camera.CAMERAS['forward']
    scenes = [synthetic.make_scene('lifting_4-small_divider', 680 + e) for e in range(2)]
    b = batch.StateBatch(scenes)
    b.enable_receptacle_cache()
    rs = np.random.RandomState(3)
    tgt = np.stack([rs.uniform(-0.3, 0.3, (b.N, 40)), rs.uniform(-0.3, 0.3, (b.N, 40))], -1)
    f = [synthetic.camera_images(scenes[e], a, 'forward', seed=200 + 7 * e + a) for e, a in b.agents]
    prep = b.prepare_ingest(np.stack([x[0] for x in f]), np.stack([x[1] for x in f]).astype(np.int32))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.launch_ingest(prep)
    assert b._replayed.all()
    b.render()                       # fills the cache from the (not yet replayed) maps
    torch.cuda.synchronize()
    g.replay()                       # the maps change; no host version moves
    torch.cuda.synchronize()
    for n, (e, a) in enumerate(b.agents):
        r = scenes[e]['robots'][a]
        O.ingest(scenes[e]['overhead'][a], scenes[e]['occupancy'][a], f[n][0], f[n][1].astype(np.int32),
                 spec.params(r['position'][0], r['position'][1], r['heading']), spec, synthetic.SEG_IDS,
                 scenes[e]['receptacle_position'] is not None)
    _rec_check(b, scenes, tgt, 'after replay')
    _rec_check(b, scenes, tgt, 'again')  # still a miss: the next replay may change the maps again


def test_receptacle_cache_across_streams(V):
    """the receptacle cache is written by render() and the miss path and read by
    the lookups; a launch on another stream than the last cache user's waits for an event recorded
    on that stream (on the same stream, stream order suffices).  A render
    on a side stream followed at once by lookups on the current stream (and the other way round)
    equals the oracle."""
    synthetic, vector_env = V
    from simaps import batch
    scenes = [synthetic.make_scene('lifting_4-small_divider', 690 + e) for e in range(16)]
    b = batch.StateBatch(scenes)
    b.enable_receptacle_cache()
    rs = np.random.RandomState(4)
    tgt = np.stack([rs.uniform(-0.3, 0.3, (b.N, 24)), rs.uniform(-0.3, 0.3, (b.N, 24))], -1)
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    side_out = b.render(stream=side)
    assert b._rec_stream == side and (b._rec_ver == b._map_ver).all()
    _rec_check(b, scenes, tgt, 'render on side, lookup on current')
    out = b.receptacle_distances(tgt, stream=side)   # lookups on the side stream ...
    b.render()                                       # ... then a render on the current one
    torch.cuda.current_stream().wait_stream(side)
    _rec_check(b, scenes, tgt, 'after both')
    torch.cuda.synchronize()
    assert side_out.shape[0] == b.N and out.shape == (b.N, 24)


def test_distance_to_receptacle_dropin(V):
    synthetic, vector_env = V
    scenes = [synthetic.make_scene('lifting_2_throwing_2-large_empty', 70 + e) for e in range(3)]
    obs = vector_env.VectorEnvObservations(scenes)
    rs = np.random.RandomState(5)
    pos = [[[tuple(rs.uniform(-0.55, 0.55, 2)) + (0.0,) for _ in range(rs.randint(0, 7))] for _ in s['robots']]
           for s in scenes]
    got = obs.distance_to_receptacle(pos)
    for e, s in enumerate(scenes):
        for a in range(len(s['robots'])):
            ao = O.AgentOracle(s, a)
            assert got[e][a] == [ao.shortest_path_distance(s['receptacle_position'], p) for p in pos[e][a]]


@pytest.fixture(params=[1, 2, 3], ids=['compact', 'early_exit', 'overlap'])
def path_mode(request):
    """Every path kernel variant (include/simaps.h simaps_path_mode): 1 the SPFA to an empty queue,
    2 the SSSP fixpoint first and the SPFA only until the target's parent chain is final, 3 the same
    early exit with the fixpoint's sweeps running beside the SPFA (fixpoint in LDS)."""
    from simaps import _lib
    prev = _lib.lib.simaps_path_mode(request.param)
    yield request.param
    _lib.lib.simaps_path_mode(prev)


def test_shortest_path_reference_goldens(V, path_mode):
    """Movement paths through simaps_shortest_path vs the reference's own
    OccupancyMap.shortest_path outputs (straight-line test, EDT snap, exact SPFA parents,
    approximate_polygon, line-of-sight pruning)."""
    synthetic, vector_env = V
    from simaps import batch
    z = G.load('paths.npz')
    groups = {}
    for k in z.files:
        if not k.endswith('_path') or k.startswith('demo'):
            continue
        key = k[:-len('_path')]
        head, q = key.rsplit('_q', 1)
        cfg, rest = head.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        groups.setdefault(cfg, []).append((e, a, key))
    nontrivial = 0
    for cfg, items in groups.items():
        scenes = [synthetic.make_scene(cfg, 60 + e) for e in range(2)]
        b = batch.StateBatch(scenes)
        slots = [b.agents.index((e, a)) for e, a, _ in items]
        got = b.shortest_paths(np.stack([z[k + '_src'] for _, _, k in items]),
                               np.stack([z[k + '_tgt'] for _, _, k in items]), slots=slots)
        for (e, a, key), path in zip(items, got):
            want = z[key + '_path']
            nontrivial += len(want) > 2
            assert np.array_equal(np.array([p[:2] for p in path]), want), key
    assert nontrivial >= 40


def test_dropin_shortest_path_reference_goldens(V):
    """VectorEnvObservations.shortest_path (Mapper.shortest_path, envs.py:2186-2187, as
    Robot.store_new_action calls it, 875-876) against the reference's paths.npz: the waypoints
    between the ends exactly, the caller's own source / target objects at the ends (envs.py:2486,
    2500-2503), and repeated robots in one batch."""
    synthetic, vector_env = V
    z = G.load('paths.npz')
    groups = {}
    for k in z.files:
        if not k.endswith('_path') or k.startswith('demo'):
            continue
        key = k[:-len('_path')]
        head, q = key.rsplit('_q', 1)
        cfg, rest = head.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        groups.setdefault(cfg, []).append((e, a, key))
    n = 0
    for cfg, items in groups.items():
        obs = vector_env.VectorEnvObservations([synthetic.make_scene(cfg, 60 + e) for e in range(2)])
        reqs = [((e, a), tuple(z[k + '_src'].tolist()) + (0.0123,), list(z[k + '_tgt'].tolist())) for e, a, k in items]
        got = obs.shortest_path(reqs)
        assert len(got) == len(items)
        for (e, a, key), (_, s, t), path in zip(items, reqs, got):
            want = z[key + '_path']
            assert path[0] is s and path[-1] is t, key
            assert np.array_equal(np.array([p[:2] for p in path]), want), key
            assert all(len(p) == 3 and p[2] == 0 for p in path[1:-1]), key
            n += 1
    assert n >= 200
    assert obs.shortest_path([]) == []


def test_maze_paths_reference_goldens(V, path_mode):
    """Movement paths on the maze environments (large_doors / tunnels / rooms) vs the reference's
    own OccupancyMap.shortest_path: long detours through doors and tunnels, exactly."""
    synthetic, vector_env = V
    from simaps import batch
    z = G.load('maze_paths.npz')
    groups = {}
    for k in z.files:
        if not k.endswith('_path') or k == 'longest_path':
            continue
        key = k[:-len('_path')]
        head, q = key.rsplit('_q', 1)
        cfg, rest = head.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        groups.setdefault(cfg, []).append((e, a, key))
    assert len(groups) == 3
    longest = 0
    for cfg, items in groups.items():
        scenes = [synthetic.make_scene(cfg, 70 + e, observe_all=True) for e in range(3)]
        b = batch.StateBatch(scenes)
        slots = [b.agents.index((e, a)) for e, a, _ in items]
        got = b.shortest_paths(np.stack([z[k + '_src'] for _, _, k in items]),
                               np.stack([z[k + '_tgt'] for _, _, k in items]), slots=slots)
        for (e, a, key), path in zip(items, got):
            assert np.array_equal(np.array([p[:2] for p in path]), z[key + '_path']), key
            longest = max(longest, len(path))
    assert longest == int(z['longest_path']) >= 5


def test_ingest_reference_goldens(V):
    """Observation ingest through simaps_ingest vs the reference's own
    Mapper.update on the committed frames (forward-facing and overhead cameras)."""
    synthetic, vector_env = V
    from simaps import batch
    z = G.load('ingest.npz')
    for cfg, kind in (('lifting_4-small_divider', 'forward'), ('pushing_4-large_empty', 'overhead')):
        s = synthetic.make_scene(cfg, 80)
        b = batch.StateBatch([s])
        keys = ['%s_a%d' % (cfg, a) for a in range(2)]
        b.ingest(np.stack([z[k + '_depth'] for k in keys]), np.stack([z[k + '_seg'].astype(np.int32) for k in keys]),
                 camera=kind, slots=[0, 1])
        ov, oc = b.overhead.cpu().numpy(), b.occupancy.cpu().numpy()
        for a, k in enumerate(keys):
            assert _bitwise(ov[a], z[k + '_overhead']), k
            assert np.array_equal(oc[a], z[k + '_occupancy']), k
        assert _key_epochs(b) <= {0, b._epoch}        # keys: untouched, or this (first) launch's epoch


@pytest.mark.parametrize('kind', ['forward', 'overhead'])
def test_ingest_then_get_state_vs_oracle(V, kind):
    """update_map + get_state end to end on the device vs the oracle (fresh frames; z ties resolved
    as 'later camera pixel wins' on both sides)."""
    synthetic, vector_env = V
    from simaps import batch
    scenes = [synthetic.make_scene('lifting_2_throwing_2-large_empty', 210 + e) for e in range(3)]
    b = batch.StateBatch(scenes)
    frames = [synthetic.camera_images(scenes[e], a, kind, seed=7 * e + a) for e, a in b.agents]
    b.ingest(np.stack([f[0] for f in frames]), np.stack([f[1] for f in frames]), camera=kind)
    st = b.as_hwc(b.render()).cpu().numpy()
    from simaps import camera
    spec = camera.CAMERAS[kind]
    ov, oc = b.overhead.cpu().numpy(), b.occupancy.cpu().numpy()
    for n, (e, a) in enumerate(b.agents):
        s = scenes[e]
        r = s['robots'][a]
        O.ingest(s['overhead'][a], s['occupancy'][a], frames[n][0], frames[n][1],
                 spec.params(r['position'][0], r['position'][1], r['heading']), spec, synthetic.SEG_IDS,
                 s['receptacle_position'] is not None)
        assert _bitwise(ov[n], s['overhead'][a]) and np.array_equal(oc[n], s['occupancy'][a]), (e, a)
        assert _bitwise(st[n], O.agent_state(s, a)), (e, a)


def test_ingest_full_size_two_frames_vs_oracle(V):
    """The BASELINE launch size (64 envs x 4 agents = 256 frames, 22 point chunks each) ingested
    three times in a row (each frame lands on the previous one's maps, whose keys carry an older
    epoch; the third launch wraps the epoch, so the key map is zeroed first): every agent's
    overhead / occupancy bitwise vs the oracle, and no key newer than its launch's epoch."""
    synthetic, vector_env = V
    from simaps import batch, camera
    scenes = [synthetic.make_scene('lifting_4-small_divider', 400 + e) for e in range(64)]
    b = batch.StateBatch(scenes)
    spec = camera.CAMERAS['forward']
    for rep in range(3):
        frames = [synthetic.camera_images(scenes[e], a, 'forward', seed=97 * rep + 5 * e + a) for e, a in b.agents]
        if rep == 2:
            b._epoch = 255  # the next launch wraps: zero the key map, epoch 1
        b.ingest(np.stack([f[0] for f in frames]), np.stack([f[1] for f in frames]), camera='forward')
        assert b._epoch == (rep + 1 if rep < 2 else 1)
        # keys untouched since the last zeroing, or of this or an earlier launch's epoch; after the
        # wrap only this launch's
        assert max(_key_epochs(b)) == b._epoch and (rep < 2 or _key_epochs(b) <= {0, 1})
        for n, (e, a) in enumerate(b.agents):
            s, r = scenes[e], scenes[e]['robots'][a]
            O.ingest(s['overhead'][a], s['occupancy'][a], frames[n][0], frames[n][1],
                     spec.params(r['position'][0], r['position'][1], r['heading']), spec, synthetic.SEG_IDS,
                     s['receptacle_position'] is not None)
    ov, oc = b.overhead.cpu().numpy(), b.occupancy.cpu().numpy()
    for n, (e, a) in enumerate(b.agents):
        assert _bitwise(ov[n], scenes[e]['overhead'][a]) and np.array_equal(oc[n], scenes[e]['occupancy'][a]), (e, a)


def test_ingest_graph_capture_replays(V):
    """an ingest captured into a graph replays its epoch, so it runs in the zeroing mode
    (epoch 0).  An eager launch leaves old-epoch keys, the capture then also zeroes the key map,
    replays with new frames copied into the captured inputs (and an eager launch in between, which
    now takes the zeroing mode too) all equal the oracle applied in the same order, and the key map
    is all zero after each launch."""
    synthetic, vector_env = V
    from simaps import batch, camera
    scenes = [synthetic.make_scene('lifting_4-small_divider', 620 + e) for e in range(3)]
    b = batch.StateBatch(scenes)
    spec = camera.CAMERAS['forward']

    def frames(seed):
        f = [synthetic.camera_images(scenes[e], a, 'forward', seed=seed + 5 * e + a) for e, a in b.agents]
        return np.stack([x[0] for x in f]), np.stack([x[1] for x in f]).astype(np.int32)

    def oracle_apply(dep, seg):
        for n, (e, a) in enumerate(b.agents):
            s, r = scenes[e], scenes[e]['robots'][a]
            O.ingest(s['overhead'][a], s['occupancy'][a], dep[n], seg[n],
                     spec.params(r['position'][0], r['position'][1], r['heading']), spec, synthetic.SEG_IDS,
                     s['receptacle_position'] is not None)

    def check():
        ov, oc = b.overhead.cpu().numpy(), b.occupancy.cpu().numpy()
        for n, (e, a) in enumerate(b.agents):
            assert _bitwise(ov[n], scenes[e]['overhead'][a]) and np.array_equal(oc[n], scenes[e]['occupancy'][a]), (e, a)

    d0, s0 = frames(11)
    b.ingest(d0, s0)                                    # eager, epoch 1: old-epoch keys stay
    oracle_apply(d0, s0)
    assert b._epoch == 1 and 1 in _key_epochs(b)
    d1, s1 = frames(23)
    prep = b.prepare_ingest(d1, s1)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.launch_ingest(prep)                           # captured: key map zeroing + epoch 0 launch
    assert b._epoch == 0 and b._zero_mode
    g.replay()
    torch.cuda.synchronize()
    oracle_apply(d1, s1)
    check()
    assert _key_epochs(b) == {0}
    d2, s2 = frames(37)
    b.ingest(d2, s2)                                    # eager after a capture: zeroing mode
    oracle_apply(d2, s2)
    assert b._epoch == 0 and _key_epochs(b) == {0}
    d3, s3 = frames(41)
    prep['depth'].copy_(torch.from_numpy(d3))
    prep['seg'].copy_(torch.from_numpy(s3))
    g.replay()
    torch.cuda.synchronize()
    oracle_apply(d3, s3)
    check()
    assert _key_epochs(b) == {0}


def test_ingest_epoch_under_capture_refused(V):
    """The C ABI refuses an epoch-tagged (non-zero epoch) ingest on a capturing stream
    (SIMAPS_EUNSUPPORTED, nothing launched) and accepts epoch 0."""
    synthetic, vector_env = V
    from simaps import _lib, batch
    scenes = [synthetic.make_scene('lifting_4-small_divider', 640)]
    b = batch.StateBatch(scenes)
    f = [synthetic.camera_images(scenes[0], a, 'forward', seed=a) for e, a in b.agents]
    prep = b.prepare_ingest(np.stack([x[0] for x in f]), np.stack([x[1] for x in f]).astype(np.int32))
    torch.cuda.synchronize()

    def call(epoch):
        return _lib.lib.simaps_ingest(
            b.cfg, prep['cam'], prep['n'], _lib.ptr(prep['agents']), _lib.ptr(prep['ids']), _lib.ptr(prep['params']),
            _lib.ptr(prep['depth']), _lib.ptr(prep['seg']), _lib.ptr(b.overhead), _lib.ptr(b.occupancy),
            _lib.ptr(b._keys), _lib.ptr(b._boxes), epoch, _lib.stream_handle(torch.cuda.current_stream()))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        rc_tagged = call(7)
        rc_zero = call(0)
    assert rc_tagged == _lib.EUNSUPPORTED and b'epoch' in _lib.lib.simaps_last_error()
    assert rc_zero == 0
    g.replay()
    torch.cuda.synchronize()
    assert _key_epochs(b) == {0}


def test_gridgraph_shortest_path_reference_goldens(V, path_mode):
    """GridGraph.shortest_path (pyx:121-154) on raw cells against the reference itself: the demo
    sample (free / blocked / equal ends) and random grids with free values 1, 2, 255 (line of sight
    counts any cell != 1 as blocked), blocked sources, unreachable targets."""
    synthetic, vector_env = V
    z = G.load('grid_paths.npz')
    demo = G.load('sssp.npz')['demo_cspace']
    g = vector_env.GridGraph(demo)
    keys = sorted(k[:-4] for k in z.files if k.startswith('demo_') and k.endswith('_src'))
    got = g.shortest_paths([(tuple(z[k + '_src']), tuple(z[k + '_tgt'])) for k in keys])
    for k, p in zip(keys, got):
        assert np.array_equal(np.array(p, dtype=np.int32).reshape(-1, 2), z[k + '_path']), k
    s0 = G.load('paths.npz')                                         # the 3 demo.py-sample goldens of r1
    for q in range(3):
        p = g.shortest_path(tuple(s0['demo_%d_src' % q]), tuple(s0['demo_%d_tgt' % q]))
        assert np.array_equal(np.array(p).reshape(-1, 2), s0['demo_%d_path' % q]), q
    m = 0
    while 'rand_%d_grid' % m in z.files:
        grid = z['rand_%d_grid' % m]
        gg = vector_env.GridGraph(grid)
        pairs = [(tuple(z['rand_%d_%d_src' % (m, k)]), tuple(z['rand_%d_%d_tgt' % (m, k)])) for k in range(6)]
        for k, p in enumerate(gg.shortest_paths(pairs)):
            assert np.array_equal(np.array(p, dtype=np.int32).reshape(-1, 2), z['rand_%d_%d_path' % (m, k)]), (m, k)
        m += 1
    assert m == 12


def _tie_grids(rs):
    """Random grids that stress the exact SPFA's queue order: empty and pillar lattices (many
    equal-length paths, so the parents -- and the waypoints -- depend on the SLF swaps), random
    obstacles at several densities, long corridors."""
    grids = []
    for h, w in ((44, 92), (60, 120), (92, 92), (17, 33)):
        g = np.ones((h, w), np.uint8)
        grids.append(g.copy())                                  # empty: all-tie octile paths
        p = g.copy()
        p[2::4, 2::4] = 0                                       # pillar lattice
        grids.append(p)
        for dens in (0.08, 0.25, 0.4):
            grids.append((rs.random_sample((h, w)) > dens).astype(np.uint8))
        c = g.copy()
        c[::6, 1:] = 0                                          # serpentine corridors
        c[3::12, :-1] = 1
        c[9::12, 1:] = 1
        c[::6, 0] = 1
        c[::12, -1] = 1
        grids.append(c)
    return grids


def _dp_tie(grid, src, tgt):
    """True if approximate_polygon (skimage 0.18.3, tolerance 1) on this path's dense points meets a
    floating-point tie: two candidates of a split within 1e-9 of each other, or the maximum within
    1e-9 of the tolerance.  There the reference's own choice follows the last-bit rounding of its
    host's libm sin / cos (numpy dispatches to SIMD / SVML kernels on AVX-512 hosts), so no
    implementation -- nor the reference on another host -- is pinned to one answer."""
    H, W = grid.shape
    _, par = O.spfa(grid, src)
    u, v = src[0] * W + src[1], tgt[0] * W + tgt[1]
    dense = [[v // W, v % W]]
    while v != u:
        v = int(par[v])
        if v < 0:
            break
        dense.append([v // W, v % W])
    return _dp_tie_dense(dense)


def _dp_tie_dense(dense):
    """_dp_tie on a given dense chain (target first)."""
    c = np.array(dense)
    stack = [(0, len(c) - 1)]
    while stack:
        s, e = stack.pop()
        (r0, c0), (r1, c1) = c[s], c[e]
        dr, dc = r1 - r0, c1 - c0
        ang = -np.arctan2(dr, dc)
        sd = c0 * np.sin(ang) + r0 * np.cos(ang)
        seg = c[s + 1:e]
        if len(seg) == 0:
            continue
        r, cc = seg[:, 0], seg[:, 1]
        proj = ((r - r0) * dr + (cc - c0) * dc > 0) & (-(r - r1) * dr - (cc - c1) * dc > 0)
        d = np.where(proj, np.abs(r * np.cos(ang) + cc * np.sin(ang) - sd),
                     np.minimum(np.hypot(cc - c0, r - r0), np.hypot(cc - c1, r - r1)))
        top = np.sort(d)[::-1]
        if abs(top[0] - 1.0) < 1e-9 or (len(top) > 1 and top[0] - top[1] < 1e-9 and top[0] > 1.0):
            return True
        if top[0] > 1.0:
            k = s + int(np.argmax(d)) + 1
            stack += [(k, e), (s, k)]
    return False


def test_gridgraph_paths_fuzz_vs_oracle(V, path_mode):
    """GridGraph.shortest_path / shortest_path_image on ~1,000 (grid, source, target) cases built to
    create equal-length-path ties, bitwise against the oracle's C restatement of pyx:69-154 (itself
    pinned to the reference by tests/test_oracle_golden.py): the lane-parallel SLF resolution of the
    path kernel must leave the queue order -- hence every parent -- exactly as the reference's.
    Paths whose Douglas-Peucker split meets a floating-point tie (_dp_tie: host-libm dependent in
    the reference itself) must agree everywhere but may differ; they are counted and bounded."""
    synthetic, vector_env = V
    rs = np.random.RandomState(1234)
    n_cases = n_tie = 0
    for gi, grid in enumerate(_tie_grids(rs)):
        free = np.argwhere(grid != 0)
        if len(free) < 2:
            continue
        gg = vector_env.GridGraph(grid)
        srcs = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(4)]
        for src in srcs:
            img = gg.shortest_path_image(src)
            ref = O.spfa_image(grid, src)
            assert _bitwise(np.asarray(img, dtype=np.float32), ref.astype(np.float32)), (gi, src)
            tgts = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(10)]
            got = gg.shortest_paths([(src, t) for t in tgts])
            for t, p in zip(tgts, got):
                want = O.grid_shortest_path(grid, src, t)
                n_cases += 1
                if np.array_equal(np.array(p, dtype=np.int64).reshape(-1, 2), np.array(want, dtype=np.int64).reshape(-1, 2)):
                    continue
                assert _dp_tie(grid, src, t), (gi, src, t, p, want)
                n_tie += 1
    assert n_cases >= 900 and n_tie <= n_cases // 100, (n_cases, n_tie)


def test_policy_input_from_device_stacks(V):
    """device-rendered CHW stacks through policy_input.group_batches equal
    DQNPolicy.apply_transform (ToTensor of the (96, 96, C) float32 state, policies.py:44-45) of the
    oracle's states, bitwise, batched per robot group, with no copy of the rendered tensor."""
    synthetic, vector_env = V
    from simaps import policy_input
    cfg = 'lifting_2_throwing_2-large_empty'
    scenes = [synthetic.make_scene(cfg, 610 + e) for e in range(3)]
    obs = vector_env.VectorEnvObservations(scenes, layout='chw')
    awaiting = [[True, False, True, True], [True] * 4, [False, True, False, False]]
    state = obs.get_state(awaiting=awaiting)
    for e, s in enumerate(scenes):
        groups = vector_env.robot_groups(s)
        for (idx, bt), members in zip(policy_input.group_batches(state[e]), groups):
            want = [a for j, a in enumerate(members) if awaiting[e][a]]
            assert idx == [j for j, a in enumerate(members) if awaiting[e][a]]
            if not want:
                assert bt is None
                continue
            assert bt.is_cuda and tuple(bt.shape) == (len(want), 5, 96, 96) and bt.dtype == torch.float32
            ref = torch.cat([policy_input.apply_transform(O.agent_state(s, a)) for a in want]).numpy()
            assert np.array_equal(bt.cpu().numpy().view(np.int32), ref.view(np.int32))
        # a single state is a zero-copy view of the rendered CHW tensor
        x = state[e][0][0] if state[e][0][0] is not None else state[e][0][1]
        t = policy_input.apply_transform(x)
        assert t.data_ptr() == x.data_ptr() and t.is_contiguous()


RESET_FILES = [f.rsplit('/', 1)[1] for f in G.scene_files() if '/scene_reset_' in f]


def _golden_env(z, e, key):
    """Scene of golden env e as the drop-in receives it: `key` = 'scene' (the fixture's own
    descriptor) or 'adapter' (reference_adapter.scene_from_env run on the reference's objects),
    plus every rendered agent's maps."""
    import json
    sc = json.loads(str(z['e%d_%s' % (e, key)]))
    for r in sc['robots']:
        r['position'] = tuple(r['position'])
    if sc['receptacle_position'] is not None:
        sc['receptacle_position'] = tuple(sc['receptacle_position'])
    A = len(sc['robots'])
    sc['occupancy'] = np.stack([z['e%d_a%d_occupancy' % (e, a)] for a in range(A)])
    sc['overhead'] = np.stack([z['e%d_a%d_overhead' % (e, a)] for a in range(A)])
    return sc


@pytest.mark.parametrize('name', RESET_FILES)
def test_dropin_reset_and_not_yet_acted_robots(V, name):
    """VectorEnvObservations.get_state on the reference's reset state (env 0: every robot idle,
    None paths / target, envs.py:214-222) and on the steps after it (env 1: robot 0 moving, the
    others never acted), fed the descriptor the adapter read from the reference's own objects:
    every stack bitwise equal to the reference's Mapper.get_state (tests/golden/make_goldens.py
    gen_reset).  The reset step renders the awaiting robot only (envs.py:222, 747-752)."""
    synthetic, vector_env = V
    z = G.load(name)
    scenes = [_golden_env(z, e, 'adapter') for e in range(2)]
    flags = scenes[0]['flags']
    nr = len(scenes[0]['robots'])
    obs = vector_env.VectorEnvObservations(scenes, layout='hwc')
    full = obs.get_state(all_robots=True, numpy=True)
    for e in range(2):
        for g, idx in zip(full[e], vector_env.robot_groups(scenes[e])):
            for x, a in zip(g, idx):
                ref = z['e%d_a%d_state' % (e, a)]
                if flags['use_intention_channels'] and flags['intention_channel_encoding'] == 'nonspatial':
                    assert np.abs(x - ref).max() <= 1e-7
                else:
                    assert _bitwise(x, ref), (e, a, float(np.abs(x - ref).max()))
    awaiting = [[a == 0 for a in range(nr)], [False] * nr]
    st = obs.get_state(awaiting=awaiting, numpy=True)
    first = vector_env.robot_groups(scenes[0])[0][0]
    assert st[0][0][0] is not None and first == 0
    assert all(x is None for g in st[1] for x in g)
    assert np.array_equal(st[0][0][0], full[0][0][0])


@pytest.mark.parametrize('cfg', ['lifting_4-small_divider', 'pushing_4-large_empty'])
def test_rotate_rounding_modes(V, cfg):
    """scene_rot-plain_*: every robot at a heading where the two BLAS roundings of rotate's
    out_center disagree, rendered by the reference on a plain-dgemv host.  The kernel in 'plain'
    mode is bitwise equal to the reference; in 'fma' mode it differs from it and equals the
    oracle's FMA restatement (so the switch is what makes the difference)."""
    from simaps import batch
    z = G.load('scene_rot-plain_%s.npz' % cfg)
    scenes = [_golden_env(z, e, 'scene') for e in range(2)]
    assert scenes[0]['rotate_rounding'] == 'plain'
    b = batch.StateBatch(scenes, layout='hwc')
    st = b.render().cpu().numpy()
    for n, (e, a) in enumerate(b.agents):
        assert _bitwise(st[n], z['e%d_a%d_state' % (e, a)]), (e, a)
    fma = [dict(s, rotate_rounding='fma') for s in scenes]
    bf = batch.StateBatch(fma, layout='hwc')
    sf = bf.render().cpu().numpy()
    differ = 0
    for n, (e, a) in enumerate(bf.agents):
        differ += not _bitwise(sf[n], z['e%d_a%d_state' % (e, a)])
        assert _bitwise(sf[n], O.agent_state(fma[e], a)), (e, a)
    assert differ >= len(bf.agents) // 2, differ


@pytest.mark.parametrize('cfg', ['lifting_4-small_divider', 'lifting_2_throwing_2-large_empty', 'rescue_4-small_empty',
                                 'lifting_4-large_rooms-history', 'lifting_4-small_divider-spatial'])
def test_update_arrays_matches_scene_update(V, cfg):
    """The array fast path (update_arrays: native packing, pinned one-copy upload) renders exactly
    what update(scenes) renders, over several steps (the staging ring wraps), with robots that never
    acted among them; both equal the oracle."""
    synthetic, vector_env = V
    from simaps import batch
    base = [synthetic.make_scene(cfg, 300 + e) for e in range(4)]
    a = vector_env.VectorEnvObservations(base, layout='chw')
    b = vector_env.VectorEnvObservations(base, layout='chw')
    for step in range(5):
        scenes = [synthetic.make_scene(cfg, 300 + e, seed_base=77 * step) for e in range(4)]
        for e, sc in enumerate(scenes):  # the maps stay the batch's (base scenes')
            sc['occupancy'], sc['overhead'] = base[e]['occupancy'], base[e]['overhead']
        if step % 2:
            scenes[1] = synthetic.never_acted(scenes[1])
            scenes[3] = synthetic.never_acted(scenes[3], robots=[0, 2])
        a.update(scenes=scenes)
        b.update_arrays(**batch.descriptor_arrays(scenes))
        sa = a.get_state(all_robots=True, numpy=True)
        sb = b.get_state(all_robots=True, numpy=True)
        for e in range(4):
            for ga, gb, idx in zip(sa[e], sb[e], vector_env.robot_groups(scenes[e])):
                for xa, xb, r in zip(ga, gb, idx):
                    assert _bitwise(xa, xb), (step, e, r)
                    if step in (0, 3):
                        assert _bitwise(xb, O.agent_state(scenes[e], r)), (step, e, r)


def test_periodic_remap_successive_frames(V):
    """RobotController.step's periodic update_map (envs.py:1401-1403): one moving robot's K frames,
    taken at K successive poses, ingested in K single-robot launches (each after the pose update)
    equal the oracle applying the same frames in order; the robot's next state is the oracle's."""
    synthetic, vector_env = V
    from simaps import batch, camera
    scenes = [synthetic.make_scene('lifting_4-small_divider', 330 + e) for e in range(4)]
    obs = vector_env.VectorEnvObservations(scenes, layout='hwc')
    spec = camera.CAMERAS['forward']
    e, a = 2, 1
    sc = scenes[e]
    ref_ov, ref_oc = sc['overhead'][a].copy(), sc['occupancy'][a].copy()
    x0, y0, h0 = sc['robots'][a]['position'][0], sc['robots'][a]['position'][1], sc['robots'][a]['heading']
    arrays = batch.descriptor_arrays(scenes)
    r = obs.batch._robot_off[e] + a
    for k in range(4):  # the robot drives 2 cm and turns 10 degrees per re-map
        pose = (x0 + 0.02 * k * np.cos(h0), y0 + 0.02 * k * np.sin(h0), h0 + np.radians(10) * k)
        arrays['pose'][r] = pose
        obs.update_arrays(**arrays)
        moved = dict(sc, robots=[dict(rb) for rb in sc['robots']])
        moved['robots'][a]['position'] = (pose[0], pose[1], 0)
        moved['robots'][a]['heading'] = pose[2]
        db, raw = synthetic.camera_images(moved, a, 'forward', seed=900 + k)
        obs.update_map([(e, a)], db[None], raw[None])
        O.ingest(ref_ov, ref_oc, db, raw, spec.params(*pose), spec, synthetic.SEG_IDS, True)
    slot = obs.slot[(e, a)]
    assert _bitwise(obs.batch.overhead[slot].cpu().numpy(), ref_ov)
    assert np.array_equal(obs.batch.occupancy[slot].cpu().numpy(), ref_oc)
    # the other robots' maps are untouched
    for (e2, a2), s2 in obs.slot.items():
        if (e2, a2) != (e, a):
            assert np.array_equal(obs.batch.occupancy[s2].cpu().numpy(), scenes[e2]['occupancy'][a2])
    moved['overhead'] = sc['overhead'].copy()
    moved['occupancy'] = sc['occupancy'].copy()
    moved['overhead'][a], moved['occupancy'][a] = ref_ov, ref_oc
    st = obs.get_state(awaiting=[[False] * 4, [False] * 4, [k == a for k in range(4)], [False] * 4], numpy=True)
    g = [gi for gi, grp in enumerate(vector_env.robot_groups(sc)) if a in grp][0]
    x = st[e][g][vector_env.robot_groups(sc)[g].index(a)]
    assert _bitwise(x, O.agent_state(moved, a))


def test_path_launch_in_graph_capture(V):
    """Path launches captured into a graph: in mode 2 the early-exit kernel gets no scratch (it is
    taken from the memory pool in stream order per eager launch) and the capture runs the compact
    kernel; in the automatic mode a launch this small takes the overlapped kernel, whose fixpoint
    lives in LDS, so the capture keeps the early exit.  Every replay equals the eager launches of
    every kernel, for targets across the divider (detours: the SPFA runs)."""
    synthetic, _ = V
    from simaps import _lib, batch
    scenes = [synthetic.make_scene('lifting_4-small_divider', 70 + e) for e in range(8)]
    b = batch.StateBatch(scenes)
    rs = np.random.RandomState(3)
    rl, rw = scenes[0]['room_length'], scenes[0]['room_width']
    psrc = np.array([scenes[e]['robots'][a]['position'][:2] for e, a in b.agents])
    ptgt = np.stack([rs.uniform(0.05, rl / 2, b.N) * -np.sign(psrc[:, 0]), rs.uniform(-rw / 2, rw / 2, b.N)], -1)
    src, tgt = torch.as_tensor(psrc).cuda(), torch.as_tensor(ptgt).cuda()
    prev = _lib.lib.simaps_path_mode(0)
    try:
        eager = {}
        for mode in (1, 2, 3, 0):
            _lib.lib.simaps_path_mode(mode)
            xy, cnt = b.launch_shortest_paths(src, tgt)
            eager[mode] = (xy.cpu().numpy(), cnt.cpu().numpy())
        captured = {}
        for mode in (0, 2):
            _lib.lib.simaps_path_mode(mode)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                gxy, gcnt = b.launch_shortest_paths(src, tgt)
            gxy.fill_(np.nan)
            g.replay()
            torch.cuda.synchronize()
            _lib.check_faults()
            captured[mode] = (gxy.cpu().numpy(), gcnt.cpu().numpy())
    finally:
        _lib.lib.simaps_path_mode(prev)
    for got in captured.values():
        for xy, cnt in eager.values():
            assert np.array_equal(cnt, got[1])
            for n, c in enumerate(cnt):
                assert c >= 2 and np.array_equal(xy[n, :c], got[0][n, :c]), n
        assert (got[1] > 2).sum() >= 8  # detours


def test_path_scratch_growth(V):
    """The early-exit kernels' fixpoint scratch (stream-ordered pool memory per launch) follows the
    launch size (a small launch first, then one ~30x larger on the same stream, then the small one
    again): every launch equals the compact kernel's paths."""
    synthetic, _ = V
    from simaps import _lib, batch
    scenes = [synthetic.make_scene('lifting_4-small_divider', 300 + e) for e in range(80)]
    b = batch.StateBatch(scenes)
    rs = np.random.RandomState(5)
    rl, rw = scenes[0]['room_length'], scenes[0]['room_width']
    psrc = np.array([scenes[e]['robots'][a]['position'][:2] for e, a in b.agents])
    ptgt = np.stack([rs.uniform(0.05, rl / 2, b.N) * -np.sign(psrc[:, 0]), rs.uniform(-rw / 2, rw / 2, b.N)], -1)
    prev = _lib.lib.simaps_path_mode(1)
    try:
        want = b.shortest_paths(psrc, ptgt)
        _lib.lib.simaps_path_mode(2)
        for n in (10, b.N, 10):
            got = b.shortest_paths(psrc[:n], ptgt[:n], slots=list(range(n)))
            assert got == want[:n], n
    finally:
        _lib.lib.simaps_path_mode(prev)
    assert sum(len(p) > 2 for p in want) >= 50  # detours: the SPFA runs
