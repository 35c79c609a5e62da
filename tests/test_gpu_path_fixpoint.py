"""GPU tests of the opt-in fixpoint-parent path modes (simaps_path_mode 4 / 5).

These modes run no SPFA: the target's chain is walked on the f32 fixpoint of the directional sweeps
(parent of v = a neighbour u with fl(D(u) + w) == D(v); ties: smallest D(u), then pyx:30 edge order
(4), or edge order alone (5)), then approximate_polygon and the line-of-sight pruning of pyx:141-152.
The chain is a different rule from the reference's (its SPFA's parents), so these paths are checked
bitwise against the ORACLE's restatement of the same rule (oracle.fixpoint_chain), not against the
reference's goldens; how close they come to the reference's paths is measured in tools/path_modes.py
(DESIGN.md section 5).  As for the exact modes, a path whose Douglas-Peucker split meets a
floating-point tie may differ (host / device libm); those are counted and bounded.
"""
import numpy as np
import pytest
import torch

import goldens as G
import oracle as O
from test_gpu_dropin import _dp_tie_dense, _tie_grids

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def V():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a GPU (run with -m gpu on an MI355X)')
    from simaps import synthetic, vector_env
    return synthetic, vector_env


@pytest.fixture(params=[4, 5], ids=['fixpoint_min', 'fixpoint_edge'])
def rule(request):
    from simaps import _lib
    prev = _lib.lib.simaps_path_mode(request.param)
    yield request.param - 3  # oracle.fixpoint_chain rule 1 / 2
    _lib.lib.simaps_path_mode(prev)


def _same(p, q):
    return np.array_equal(np.asarray(p, dtype=np.float64).reshape(-1, 2), np.asarray(q, dtype=np.float64).reshape(-1, 2))


def test_gridgraph_fixpoint_paths_vs_oracle(V, rule):
    """~1,000 GridGraph.shortest_path cases on the tie-heavy grids (empty / pillar lattices, random
    obstacles, corridors), LDS-resident windows: bitwise the oracle's fixpoint-rule paths."""
    synthetic, vector_env = V
    rs = np.random.RandomState(4321)
    n_cases = n_tie = n_detour = 0
    for gi, grid in enumerate(_tie_grids(rs)):
        free = np.argwhere(grid != 0)
        if len(free) < 2:
            continue
        gg = vector_env.GridGraph(grid)
        for _ in range(4):
            src = tuple(int(x) for x in free[rs.randint(len(free))])
            tgts = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(10)]
            got = gg.shortest_paths([(src, t) for t in tgts])
            for t, p in zip(tgts, got):
                want = O.grid_shortest_path(grid, src, t, fixpoint_rule=rule)
                n_cases += 1
                n_detour += len(want) > 2
                if _same(p, want):
                    continue
                assert _dp_tie_dense(O.fixpoint_chain(grid, src, t, rule)), (gi, src, t, p, want)
                n_tie += 1
    assert n_cases >= 900 and n_detour >= 300
    assert n_tie <= n_cases // 100


def test_gridgraph_fixpoint_paths_large_window(V, rule):
    """The demo.py sample with the whole 232 x 232 grid as the window (the global-memory kernels of
    csrc/grid_large.h, gl_path_kernel's fixp walk) against the oracle; an unreachable / blocked
    target gives [target]."""
    synthetic, vector_env = V
    from simaps import batch
    demo = G.load('sssp.npz')['demo_cspace']
    H, W = demo.shape
    z = G.load('grid_paths.npz')
    keys = sorted(k[:-4] for k in z.files if k.startswith('demo_') and k.endswith('_src'))
    pairs = [(tuple(int(x) for x in z[k + '_src']), tuple(int(x) for x in z[k + '_tgt'])) for k in keys]
    blocked = tuple(int(x) for x in np.argwhere(demo == 0)[0])
    pairs.append((pairs[0][0], blocked))
    g = torch.from_numpy(demo).cuda().unsqueeze(0).expand(len(pairs), H, W).contiguous()
    got = batch.grid_paths(g, [p[0] for p in pairs], [p[1] for p in pairs], window=(0, 0, H, W), max_points=512)
    for (s, t), p in zip(pairs, got):
        want = O.grid_shortest_path(demo, s, t, fixpoint_rule=rule)
        assert _same(p, want) or _dp_tie_dense(O.fixpoint_chain(demo, s, t, rule)), (s, t, p, want)
    assert _same(got[-1], [blocked])


def test_movement_fixpoint_paths_vs_oracle(V, rule):
    """OccupancyMap.shortest_path (simaps_shortest_path) at the reference fixtures' sources and targets
    (paths.npz: straight lines, snapped ends, detours around the divider) and fresh ones: bitwise the
    oracle's AgentOracle.shortest_path with the same rule."""
    synthetic, vector_env = V
    from simaps import batch
    z = G.load('paths.npz')
    groups = {}
    for k in z.files:
        if not k.endswith('_path') or k.startswith('demo'):
            continue
        key = k[:-len('_path')]
        head, _ = key.rsplit('_q', 1)
        cfg, rest = head.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        groups.setdefault(cfg, []).append((e, a, key))
    n = n_tie = n_detour = 0
    for cfg, items in groups.items():
        scenes = [synthetic.make_scene(cfg, 60 + e) for e in range(2)]
        b = batch.StateBatch(scenes)
        rs = np.random.RandomState(len(cfg))
        rl, rw = scenes[0]['room_length'], scenes[0]['room_width']
        extra = [(e, a, rs.uniform(-rl / 2 + 0.02, rl / 2 - 0.02), rs.uniform(-rw / 2 + 0.02, rw / 2 - 0.02))
                 for e, a in b.agents for _ in range(3)]
        srcs = [z[k + '_src'] for _, _, k in items] + [np.array(scenes[e]['robots'][a]['position'][:2]) for e, a, _, _ in extra]
        tgts = [z[k + '_tgt'] for _, _, k in items] + [np.array([x, y]) for _, _, x, y in extra]
        who = [(e, a) for e, a, _ in items] + [(e, a) for e, a, _, _ in extra]
        got = b.shortest_paths(np.stack(srcs), np.stack(tgts), slots=[b.agents.index(w) for w in who])
        oracles = {}
        for (e, a), s, t, p in zip(who, srcs, tgts, got):
            ao = oracles.setdefault((e, a), O.AgentOracle(scenes[e], a))
            want = ao.shortest_path(s, t, fixpoint_rule=rule)
            n += 1
            n_detour += len(want) > 2
            if _same([q[:2] for q in p], want):
                continue
            assert _dp_tie_dense(O.fixpoint_chain(ao.cspace, ao.snap(s), ao.snap(t), rule)), (cfg, e, a, s, t)
            n_tie += 1
    assert n >= 400 and n_detour >= 80
    assert n_tie <= max(2, n // 100)


def test_fixpoint_mode_keeps_lookups_and_states(V):
    """The path mode only changes the movement-path kernels: reward lookups and rendered states are
    unchanged bit for bit."""
    synthetic, vector_env = V
    from simaps import _lib, batch
    scenes = [synthetic.make_scene('lifting_4-small_divider', 77 + e) for e in range(2)]
    b = batch.StateBatch(scenes)
    src = np.array([scenes[e]['robots'][a]['position'][:2] for e, a in b.agents])
    tgt = src[:, None, :] + np.array([[0.3, 0.1], [-0.2, 0.05]])[None]
    ref_states = b.render().cpu().numpy()
    ref_d = b.shortest_path_distances(src, tgt).cpu().numpy()
    prev = _lib.lib.simaps_path_mode(4)
    try:
        st = b.render().cpu().numpy()
        d = b.shortest_path_distances(src, tgt).cpu().numpy()
    finally:
        _lib.lib.simaps_path_mode(prev)
    assert np.array_equal(st.view(np.int32), ref_states.view(np.int32))
    assert np.array_equal(d, ref_d)
