"""GPU tests of the always-on device fault path (include/simaps.h SIMAPS_FAULT_*) and of launches
on a side stream.

A kernel that hits a condition invalidating its output -- a wave-group barrier that gave up
waiting, the SSSP round cap, or a descriptor field clamped to this build's limits -- posts a bit
to the library's host-mapped fault word.  simaps_fault_status reads it after a sync, and the next
compute call fails with SIMAPS_EDEVICE, with or without debug buffers.
"""
import os

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG_LIB = os.path.join(ROOT, 'spatial-intention-maps_amd', 'simaps', 'libsimaps_diagflag.so')
DIAG_RING_LIB = os.path.join(ROOT, 'spatial-intention-maps_amd', 'simaps', 'libsimaps_diagring.so')


@pytest.fixture(scope='module')
def S():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a GPU (run with -m gpu on an MI355X)')
    from simaps import _lib, batch, synthetic
    _lib.lib.simaps_fault_status(1)
    yield _lib, batch, synthetic
    _lib.lib.simaps_fault_status(1)


def _launch(L, _lib, b, robots_d, envs_d, agents_d, paths_d, out, n):
    return L.simaps_get_state(b.cfg, n, _lib.ptr(agents_d), _lib.ptr(envs_d), _lib.ptr(robots_d), _lib.ptr(paths_d),
                              _lib.ptr(b.occupancy), _lib.ptr(b.overhead), _lib.ptr(out), 0, None,
                              _lib.stream_handle())


def _dev(batch, a, device):
    return batch._to_dev(a, device)


def test_clean_run_posts_no_fault(S):
    _lib, batch, synthetic = S
    b = batch.StateBatch([synthetic.make_scene('lifting_4-small_divider', e) for e in range(8)])
    b.render()
    torch.cuda.synchronize()
    assert _lib.lib.simaps_fault_status(0) == 0
    _lib.check_faults()


@pytest.mark.parametrize('bad', ['num_robots', 'robot_index', 'path_length'])
def test_descriptor_clamp_is_reported(S, bad):
    """num_robots > SIMAPS_MAX_ROBOTS, a robot index past num_robots, or an intention path longer
    than SIMAPS_MAX_PATH: the kernel clamps (no out-of-range LDS access) and reports it."""
    _lib, batch, synthetic = S
    scene = synthetic.make_scene('lifting_4-small_divider', 5)
    b = batch.StateBatch([scene])
    robots, envs, ag, paths = batch.pack_descriptors([scene], b.agents)
    robots = np.concatenate([robots, np.repeat(robots[:1], 8)])       # records past num_robots exist
    paths = np.concatenate([paths, np.repeat(paths[:1], 40, 0)])
    if bad == 'num_robots':
        envs['num_robots'] = 9
    elif bad == 'robot_index':
        ag['robot'][1] = 6
    else:
        robots['intention_len'][2] = 17
    out = b.alloc_state()
    dev = lambda a: _dev(batch, a, b.device)  # noqa: E731
    R, E, A, P = dev(robots), dev(envs), dev(ag), torch.from_numpy(paths).to(b.device)
    assert _launch(_lib.lib, _lib, b, R, E, A, P, out, b.N) == 0
    torch.cuda.synchronize()
    assert _lib.lib.simaps_fault_status(0) == _lib.FAULT_DESCRIPTOR
    # the next compute call refuses once (and clears the word), then works again
    assert _launch(_lib.lib, _lib, b, R, E, A, P, out, b.N) == _lib.EDEVICE
    assert b'descriptor clamped' in _lib.lib.simaps_last_error()
    torch.cuda.synchronize()
    _lib.lib.simaps_fault_status(1)
    b.render()
    torch.cuda.synchronize()
    assert _lib.lib.simaps_fault_status(0) == 0


def test_barrier_timeout_flag_reaches_the_caller(S):
    """Diagnostic build libsimaps_diagflag.so raises the barrier-timeout flag at its real site (the
    Group::sync spin) but keeps waiting: the output is still exact, and the fault surfaces through
    simaps_fault_status, the next call's SIMAPS_EDEVICE, and simaps._lib.check_faults."""
    _lib, batch, synthetic = S
    if not os.path.exists(DIAG_LIB):
        pytest.fail('build the diagnostic library first: make -C spatial-intention-maps_amd/csrc diag')
    L = _lib._load(DIAG_LIB)
    scenes = [synthetic.make_scene('lifting_4-small_divider', 40 + e) for e in range(4)]
    b = batch.StateBatch(scenes)
    assert L.simaps_fault_status(1) == 0
    out = b.alloc_state()
    assert _launch(L, _lib, b, b.robots_d, b.envs_d, b.agents_d, b.paths_d, out, b.N) == 0
    st = b.as_hwc(out).cpu().numpy()
    assert L.simaps_fault_status(0) & _lib.FAULT_TIMEOUT
    # the next call refuses (and clears the word); a new launch posts the flag again
    assert _launch(L, _lib, b, b.robots_d, b.envs_d, b.agents_d, b.paths_d, out, b.N) == _lib.EDEVICE
    assert L.simaps_fault_status(0) == 0
    assert _launch(L, _lib, b, b.robots_d, b.envs_d, b.agents_d, b.paths_d, out, b.N) == 0
    torch.cuda.synchronize()
    with pytest.raises(_lib.DeviceFault):
        _lib.check_faults(L)
    assert L.simaps_fault_status(0) == 0
    for n, (e, a) in enumerate(b.agents):
        assert np.array_equal(st[n].view(np.int32), O.agent_state(scenes[e], a).view(np.int32))
    assert _lib.lib.simaps_fault_status(0) == 0       # the product library's word is separate


def test_path_pop_cap_reaches_the_caller(S):
    """the path kernels post SIMAPS_FAULT_ROUNDS when the SPFA's pop guard stops a live
    queue (the diagnostic build caps it at 64 pops, which every detour query exceeds), so a capped
    run cannot return wrong waypoints with rc 0; straight-line queries (no SPFA) post nothing."""
    _lib, batch, synthetic = S
    if not os.path.exists(DIAG_LIB):
        pytest.fail('build the diagnostic library first: make -C spatial-intention-maps_amd/csrc diag')
    L = _lib._load(DIAG_LIB)
    L.simaps_fault_status(1)
    scene = synthetic.make_scene('lifting_4-small_divider', 3)
    b = batch.StateBatch([scene])
    rl, rw = scene['room_length'], scene['room_width']

    def run(src, tgt):
        s = torch.tensor(src, dtype=torch.float64, device=b.device)
        t = torch.tensor(tgt, dtype=torch.float64, device=b.device)
        xy = torch.empty((b.N, 64, 2), dtype=torch.float64, device=b.device)
        cnt = torch.empty((b.N,), dtype=torch.int32, device=b.device)
        rc = L.simaps_shortest_path(b.cfg, b.N, _lib.ptr(b.agents_d), _lib.ptr(b.envs_d), _lib.ptr(b.robots_d),
                                    _lib.ptr(b.occupancy), _lib.ptr(s), _lib.ptr(t), 64, _lib.ptr(xy), _lib.ptr(cnt),
                                    _lib.stream_handle())
        torch.cuda.synchronize()
        return rc
    # across the divider: every query needs a detour (SPFA)
    src = [[-rl / 4, -rw / 4]] * b.N
    tgt = [[rl / 4, rw / 4 - 0.01 * a] for a in range(b.N)]
    assert run(src, tgt) == 0
    assert L.simaps_fault_status(0) & _lib.FAULT_ROUNDS
    with pytest.raises(_lib.DeviceFault):
        _lib.check_faults(L)
    # a straight line (same point) runs no SPFA: no fault
    assert run(src, src) == 0
    assert L.simaps_fault_status(0) == 0
    assert _lib.lib.simaps_fault_status(0) == 0


def test_large_grid_pop_cap_scales_with_the_window(S):
    """the large-grid path kernel's pop guard is max(SIMAPS_POP_CAP, 8 V + 1) -- the
    reference's linear queue holds 8 V entries (pyx:78), so no SPFA it can run pops more.  The
    diagnostic build lowers the constant to 64, which every query below exceeds: the scaled cap,
    not the constant, must apply -- exact reference paths and no fault.  Unreachable and blocked
    targets skip the SPFA and give [target]."""
    _lib, batch, synthetic = S
    if not os.path.exists(DIAG_LIB):
        pytest.fail('build the diagnostic library first: make -C spatial-intention-maps_amd/csrc diag')
    import goldens as G
    L = _lib._load(DIAG_LIB)
    L.simaps_fault_status(1)
    demo = G.load('sssp.npz')['demo_cspace']
    H, W = demo.shape
    z = G.load('grid_paths.npz')
    keys = sorted(k[:-4] for k in z.files if k.startswith('demo_') and k.endswith('_src'))
    blocked = tuple(int(x) for x in np.argwhere(demo == 0)[0])
    srcs = [tuple(z[k + '_src']) for k in keys] + [tuple(z[keys[0] + '_src'])]
    tgts = [tuple(z[k + '_tgt']) for k in keys] + [blocked]
    B = len(srcs)
    g = torch.from_numpy(demo).cuda().unsqueeze(0).expand(B, H, W).contiguous()
    src = torch.tensor(srcs, dtype=torch.int32, device='cuda')
    tgt = torch.tensor(tgts, dtype=torch.int32, device='cuda')
    ij = torch.empty((B, 512, 2), dtype=torch.int32, device='cuda')
    cnt = torch.empty((B,), dtype=torch.int32, device='cuda')
    rc = L.simaps_grid_path(B, H, W, _lib.ptr(g), _lib.ptr(src), _lib.ptr(tgt), 0, 0, H, W, 512, _lib.ptr(ij),
                            _lib.ptr(cnt), _lib.stream_handle())
    torch.cuda.synchronize()
    assert rc == 0
    assert L.simaps_fault_status(0) == 0
    ij, cnt = ij.cpu().numpy(), cnt.cpu().numpy()
    for q, k in enumerate(keys):
        assert np.array_equal(ij[q, :cnt[q]], z[k + '_path']), k
    assert cnt[-1] == 1 and tuple(ij[-1, 0]) == blocked
    assert _lib.lib.simaps_fault_status(0) == 0


def test_overlap_sweep_barrier_flag_reaches_the_caller(S):
    """The overlapped path kernel (simaps_path_mode 3) separates its sweep rounds with a 3-wave
    Group barrier; the diagnostic build raises the barrier-timeout flag at that spin too, and it
    surfaces like get_state's.  Straight-line queries run neither sweeps nor SPFA: no flag."""
    _lib, batch, synthetic = S
    if not os.path.exists(DIAG_LIB):
        pytest.fail('build the diagnostic library first: make -C spatial-intention-maps_amd/csrc diag')
    L = _lib._load(DIAG_LIB)
    L.simaps_fault_status(1)
    prev = L.simaps_path_mode(3)
    try:
        scene = synthetic.make_scene('lifting_4-small_divider', 5)
        b = batch.StateBatch([scene])
        rl, rw = scene['room_length'], scene['room_width']

        def run(src, tgt):
            s = torch.tensor(src, dtype=torch.float64, device=b.device)
            t = torch.tensor(tgt, dtype=torch.float64, device=b.device)
            xy = torch.empty((b.N, 64, 2), dtype=torch.float64, device=b.device)
            cnt = torch.empty((b.N,), dtype=torch.int32, device=b.device)
            rc = L.simaps_shortest_path(b.cfg, b.N, _lib.ptr(b.agents_d), _lib.ptr(b.envs_d), _lib.ptr(b.robots_d),
                                        _lib.ptr(b.occupancy), _lib.ptr(s), _lib.ptr(t), 64, _lib.ptr(xy),
                                        _lib.ptr(cnt), _lib.stream_handle())
            torch.cuda.synchronize()
            return rc
        src = [[-rl / 4, -rw / 4]] * b.N
        assert run(src, [[rl / 4, rw / 4 - 0.01 * a] for a in range(b.N)]) == 0
        assert L.simaps_fault_status(0) & _lib.FAULT_TIMEOUT
        with pytest.raises(_lib.DeviceFault):
            _lib.check_faults(L)
        assert run(src, src) == 0
        assert L.simaps_fault_status(0) == 0
    finally:
        L.simaps_path_mode(prev)
    assert _lib.lib.simaps_fault_status(0) == 0


@pytest.mark.parametrize('mode', [1, 2, 3], ids=['compact', 'early_exit', 'overlap'])
def test_spfa_ring_wraps_exact(S, monkeypatch, mode):
    """The product SPFA's queue ring has one slot per room cell, and a query pops about once per
    free cell, so its wrap arithmetic rarely runs.  The diagnostic ring build (libsimaps_diagring.so,
    SIMAPS_SPFA_RING=521) caps the ring at 521 slots: every query of more than 521 pops -- the
    large-room maze detours pop ~6,500 -- wraps it many times.  The reference's own movement and
    maze paths and the grid-path fuzz cases must stay exact, and the ring must never overflow."""
    _lib, batch, synthetic = S
    if not os.path.exists(DIAG_RING_LIB):
        pytest.fail('build the diagnostic libraries first: make -C spatial-intention-maps_amd/csrc diag')
    import goldens as G
    from test_gpu_dropin import _dp_tie, _tie_grids
    from simaps import vector_env
    L = _lib._load(DIAG_RING_LIB)
    L.simaps_fault_status(1)
    prev = L.simaps_path_mode(mode)
    monkeypatch.setattr(_lib, 'lib', L)   # the package's entry points call _lib.lib at call time
    try:
        for name, seed0, observe_all in (('maze_paths.npz', 70, True), ('paths.npz', 60, False)):
            z = G.load(name)
            groups = {}
            for k in z.files:
                if not k.endswith('_path') or k.startswith('demo') or k == 'longest_path':
                    continue
                key = k[:-len('_path')]
                cfg, rest = key.rsplit('_q', 1)[0].rsplit('_e', 1)
                groups.setdefault(cfg, []).append((tuple(int(x) for x in rest.split('_a')), key))
            for cfg, items in groups.items():
                scenes = [synthetic.make_scene(cfg, seed0 + e, observe_all=observe_all) for e in range(3)]
                b = batch.StateBatch(scenes)
                got = b.shortest_paths(np.stack([z[k + '_src'] for _, k in items]),
                                       np.stack([z[k + '_tgt'] for _, k in items]),
                                       slots=[b.agents.index(ea) for ea, _ in items])
                for (_, key), path in zip(items, got):
                    assert np.array_equal(np.array([p[:2] for p in path]), z[key + '_path']), (name, key)
        rs = np.random.RandomState(4321)
        for gi, grid in enumerate(_tie_grids(rs)):
            free = np.argwhere(grid != 0)
            gg = vector_env.GridGraph(grid)
            src = tuple(int(x) for x in free[rs.randint(len(free))])
            tgts = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(8)]
            for t, p in zip(tgts, gg.shortest_paths([(src, t) for t in tgts])):
                want = O.grid_shortest_path(grid, src, t)
                if not np.array_equal(np.array(p, dtype=np.int64).reshape(-1, 2), np.array(want, dtype=np.int64).reshape(-1, 2)):
                    assert _dp_tie(grid, src, t), (gi, src, t)
        torch.cuda.synchronize()
        assert L.simaps_fault_status(0) == 0   # the 521-slot ring never held more live entries
    finally:
        L.simaps_path_mode(prev)


def test_path_bad_descriptor_is_reported(S):
    """sp_distance / path kernels clamp a robot index past num_robots (and a robot class
    outside 0..3) like get_state and post SIMAPS_FAULT_DESCRIPTOR."""
    _lib, batch, synthetic = S
    scene = synthetic.make_scene('lifting_4-small_divider', 5)
    b = batch.StateBatch([scene])
    robots, envs, ag, paths = batch.pack_descriptors([scene], b.agents)
    robots = np.concatenate([robots, np.repeat(robots[:1], 8)])
    ag['robot'][1] = 6
    R, E, A = (_dev(batch, x, b.device) for x in (robots, envs, ag))
    src = torch.zeros((b.N, 2), dtype=torch.float64, device=b.device)
    tgt = torch.zeros((b.N, 3, 2), dtype=torch.float64, device=b.device)
    out = torch.empty((b.N, 3), dtype=torch.float64, device=b.device)
    _lib.lib.simaps_fault_status(1)
    assert _lib.lib.simaps_sp_distance(b.cfg, b.N, _lib.ptr(A), _lib.ptr(E), _lib.ptr(R), _lib.ptr(b.occupancy),
                                       _lib.ptr(src), _lib.ptr(tgt), 3, _lib.ptr(out), None, _lib.stream_handle()) == 0
    torch.cuda.synchronize()
    assert _lib.lib.simaps_fault_status(1) == _lib.FAULT_DESCRIPTOR
    xy = torch.empty((b.N, 64, 2), dtype=torch.float64, device=b.device)
    cnt = torch.empty((b.N,), dtype=torch.int32, device=b.device)
    assert _lib.lib.simaps_shortest_path(b.cfg, b.N, _lib.ptr(A), _lib.ptr(E), _lib.ptr(R), _lib.ptr(b.occupancy),
                                         _lib.ptr(src), _lib.ptr(src), 64, _lib.ptr(xy), _lib.ptr(cnt),
                                         _lib.stream_handle()) == 0
    torch.cuda.synchronize()
    assert _lib.lib.simaps_fault_status(1) == _lib.FAULT_DESCRIPTOR


def test_side_stream_render_matches_default_stream(S):
    """render on a non-current stream; outputs / inputs are held for that stream and the
    reader waits for it."""
    _lib, batch, synthetic = S
    from simaps import vector_env
    scenes = [synthetic.make_scene('pushing_4-large_empty', 70 + e) for e in range(6)]
    obs = vector_env.VectorEnvObservations(scenes, layout='chw')
    ref = obs.batch.as_hwc(obs.batch.render()).cpu().numpy()
    side = torch.cuda.Stream()
    for _ in range(3):
        st = obs.get_state(all_robots=True, numpy=True, stream=side)
        for e, s in enumerate(scenes):
            for g, idx in zip(st[e], vector_env.robot_groups(s)):
                for x, a in zip(g, idx):
                    assert np.array_equal(x.view(np.int32), ref[obs.slot[(e, a)]].view(np.int32))
    out = obs.batch.render(stream=side)
    torch.cuda.current_stream().wait_stream(side)
    assert np.array_equal(obs.batch.as_hwc(out).cpu().numpy().view(np.int32), ref.view(np.int32))


def test_gridgraph_side_stream_cache(S):
    """GridGraph images computed on a side stream are cached and read back on the current stream."""
    _lib, batch, synthetic = S
    from simaps import vector_env
    import goldens as G
    g = G.load('sssp.npz')
    gg = vector_env.GridGraph(g['demo_cspace'])
    side = torch.cuda.Stream()
    srcs = [(75, 156)] + [tuple(int(x) for x in p) for p in g['demo_sources']]
    imgs = gg.shortest_path_images(srcs, stream=side)
    assert np.array_equal(imgs[0].cpu().numpy().view(np.int32), g['demo_image'].view(np.int32))
    assert gg.shortest_path_distance((75, 156), (131, 112)) == float(g['demo_distance'])
    for q, s in enumerate(srcs[1:]):
        assert np.array_equal(gg.shortest_path_image(s).view(np.int32), O.spfa_image(g['demo_cspace'], s).view(np.int32))
