"""GridGraph on grids beyond the LDS-resident window: the reference's
GridGraph(grid) accepts any C-contiguous uint8 grid (shortest_paths.pyx:24-38); windows larger than
include/simaps.h's SIMAPS_MAX_ROOM_CELLS / SIMAPS_MAX_ROOM_W run the global-memory kernels of
csrc/grid_large.h.  Checked bitwise against the reference's own fixtures (the demo.py sample, run
with the whole 232 x 232 grid as the window so that the large kernels take it) and against the
oracle's C restatement of pyx:69-154 on 500 x 500 grids."""
import numpy as np
import pytest
import torch

import goldens as G
import oracle as O
from test_gpu_dropin import _bitwise, _dp_tie

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def M():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a GPU (run with -m gpu on an MI355X)')
    from simaps import batch, vector_env
    return batch, vector_env


def test_demo_sample_through_the_large_kernels(M):
    """The demo.py sample with window = the whole 232 x 232 grid (beyond SIMAPS_MAX_ROOM_W): its 12
    reference images (sha256) and the demo known answer, and its reference paths."""
    batch, vector_env = M
    import hashlib
    g = G.load('sssp.npz')
    demo = g['demo_cspace']
    H, W = demo.shape
    assert not vector_env.window_fits(H, W)
    srcs = g['demo_sources']
    grids = torch.from_numpy(demo).cuda().unsqueeze(0).expand(len(srcs), H, W).contiguous()
    imgs = batch.sssp_grid(grids, torch.from_numpy(srcs.astype(np.int32)), window=(0, 0, H, W)).cpu().numpy()
    for k in range(len(srcs)):
        assert hashlib.sha256(imgs[k].astype(np.float32).tobytes()).digest() == g['demo_sha'][k].tobytes(), k
    one = batch.sssp_grid(grids[:1], torch.tensor([[75, 156]], dtype=torch.int32), window=(0, 0, H, W)).cpu().numpy()[0]
    assert _bitwise(one, g['demo_image'])
    assert one[131, 112] == np.float32(g['demo_distance'])
    z = G.load('grid_paths.npz')
    keys = sorted(k[:-4] for k in z.files if k.startswith('demo_') and k.endswith('_src'))
    gr = torch.from_numpy(demo).cuda().unsqueeze(0).expand(len(keys), H, W).contiguous()
    got = batch.grid_paths(gr, [tuple(z[k + '_src']) for k in keys], [tuple(z[k + '_tgt']) for k in keys],
                           window=(0, 0, H, W), max_points=512)
    for k, p in zip(keys, got):
        assert np.array_equal(np.array(p, dtype=np.int32).reshape(-1, 2), z[k + '_path']), k
    s0 = G.load('paths.npz')
    got = batch.grid_paths(gr[:3], [tuple(s0['demo_%d_src' % q]) for q in range(3)],
                           [tuple(s0['demo_%d_tgt' % q]) for q in range(3)], window=(0, 0, H, W))
    for q in range(3):
        assert np.array_equal(np.array(got[q]).reshape(-1, 2), s0['demo_%d_path' % q]), q


def _big_grids(rs):
    n = 500
    yield 'rand25', (rs.random_sample((n, n)) > 0.25).astype(np.uint8)
    yield 'rand40', (rs.random_sample((n, n)) > 0.40).astype(np.uint8)      # near percolation: long detours
    e = np.ones((300, 420), np.uint8)
    e[3::5, 3::5] = 0                                                        # pillar lattice: all ties
    yield 'pillars', e
    m = np.ones((257, 300), np.uint8) * 2                                   # free value 2: line of sight blocked
    m[::8, 1:] = 0
    m[4::16, :-1] = 2
    m[::16, 0] = 2
    m[8::16, -1] = 2
    yield 'serpentine', m


def test_gridgraph_large_images_and_paths_vs_oracle(M):
    """500 x 500 random grids (two densities), a pillar lattice and a serpentine maze: the drop-in
    GridGraph takes them (no ValueError), shortest_path_image equals the oracle SPFA bitwise, and
    shortest_path equals the oracle's path (a Douglas-Peucker floating-point tie -- host-libm
    dependent in the reference itself -- may differ, counted and bounded)."""
    batch, vector_env = M
    rs = np.random.RandomState(505)
    n_cases = n_tie = 0
    for name, grid in _big_grids(rs):
        gg = vector_env.GridGraph(grid)
        assert gg.large, name
        free = np.argwhere(grid != 0)
        for _ in range(2):
            src = tuple(int(x) for x in free[rs.randint(len(free))])
            img = gg.shortest_path_image(src)
            assert _bitwise(img, O.spfa_image(grid, src)), (name, src)
            tgts = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(6)]
            got = gg.shortest_paths([(src, t) for t in tgts])
            for t, p in zip(tgts, got):
                want = O.grid_shortest_path(grid, src, t)
                n_cases += 1
                if np.array_equal(np.array(p, dtype=np.int64).reshape(-1, 2), np.array(want, dtype=np.int64).reshape(-1, 2)):
                    continue
                assert _dp_tie(grid, src, t), (name, src, t, p, want)
                n_tie += 1
            assert gg.shortest_path_distance(src, tgts[0]) == float(O.spfa_image(grid, src)[tgts[0]])
    assert n_cases == 48 and n_tie <= 2, (n_cases, n_tie)


def test_gridgraph_large_edge_cases(M):
    """Blocked source (0 at the source, -1 elsewhere), unreachable target ([target]), source ==
    target, a free region cut in two, and a 1 x 10,000 corridor (a window far beyond the LDS width)."""
    batch, vector_env = M
    rs = np.random.RandomState(7)
    grid = (rs.random_sample((200, 300)) > 0.3).astype(np.uint8)
    grid[:, 150] = 0                                                         # two halves
    gg = vector_env.GridGraph(grid)
    assert gg.large
    blocked = tuple(int(x) for x in np.argwhere(grid == 0)[5])
    assert _bitwise(gg.shortest_path_image(blocked), O.spfa_image(grid, blocked))
    a = tuple(int(x) for x in np.argwhere(grid[:, :150] != 0)[10])
    r, c = np.argwhere(grid[:, 151:] != 0)[10]
    b = (int(r), int(c) + 151)
    assert _bitwise(gg.shortest_path_image(a), O.spfa_image(grid, a))
    for s, t in ((a, b), (a, a), (blocked, a)):
        p = gg.shortest_path(s, t)
        assert np.array_equal(np.array(p).reshape(-1, 2), np.array(O.grid_shortest_path(grid, s, t)).reshape(-1, 2)), (s, t)
    corridor = np.ones((1, 10000), np.uint8)
    gc = vector_env.GridGraph(corridor)
    assert gc.large
    assert _bitwise(gc.shortest_path_image((0, 17)), O.spfa_image(corridor, (0, 17)))
    assert gc.shortest_path((0, 17), (0, 9990)) == [(0, 17), (0, 9990)]


def test_gridgraph_large_refuses_graph_capture(M):
    """The large-window kernels take their scratch in stream order per launch: under graph capture
    the C ABI refuses (SIMAPS_EUNSUPPORTED) instead of capturing an allocation."""
    batch, vector_env = M
    from simaps import _lib
    grid = torch.ones((1, 130, 130), dtype=torch.uint8, device='cuda')
    src = torch.tensor([[5, 5]], dtype=torch.int32, device='cuda')
    out = torch.empty((1, 130, 130), dtype=torch.float32, device='cuda')
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        try:
            g.capture_begin()
            rc = _lib.lib.simaps_sssp_grid(1, 130, 130, _lib.ptr(grid), _lib.ptr(src), _lib.ptr(out), 0, 0, 130, 130,
                                           _lib.stream_handle(s))
        finally:
            g.capture_end()
    assert rc == _lib.EUNSUPPORTED and b'captured' in _lib.lib.simaps_last_error()


@pytest.mark.parametrize('w', [4, 6, 9])
def test_gridgraph_large_narrow_windows(M, w):
    """Tall windows of 4, 6 and 9 columns (pitch 6, 8, 11; beyond the LDS window by their 2,000
    rows): the image and the paths equal the oracle's."""
    batch, vector_env = M
    rs = np.random.RandomState(40 + w)
    grid = (rs.random_sample((2000, w)) > 0.2).astype(np.uint8)
    gg = vector_env.GridGraph(grid)
    assert gg.large
    free = np.argwhere(grid != 0)
    src = tuple(int(x) for x in free[rs.randint(len(free))])
    assert _bitwise(gg.shortest_path_image(src), O.spfa_image(grid, src))
    tgts = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(8)]
    n_tie = 0
    for t, p in zip(tgts, gg.shortest_paths([(src, t) for t in tgts])):
        want = O.grid_shortest_path(grid, src, t)
        if not np.array_equal(np.array(p, dtype=np.int64).reshape(-1, 2), np.array(want, dtype=np.int64).reshape(-1, 2)):
            assert _dp_tie(grid, src, t), (w, src, t)
            n_tie += 1
    assert n_tie <= 1


def test_gridgraph_large_tile_seams(M):
    """The tiled fixpoint (csrc/grid_large.h gl_tile_kernel, 62 x 62 tiles): windows of whole tiles
    (124 x 186) and with one-cell partial tiles (125 x 187), sources on tile corners and seams, a
    diagonal wall that every path crosses seams along: images and paths equal the oracle's."""
    batch, vector_env = M
    rs = np.random.RandomState(62)
    for h, w in ((124, 186), (125, 187)):
        grid = (rs.random_sample((h, w)) > 0.3).astype(np.uint8)
        for k in range(min(h, w) - 20):                                          # a diagonal wall with one gap
            if k != 40:
                grid[k + 10, k + 15] = 0
        gg = vector_env.GridGraph(grid)
        assert gg.large
        for src in ((61, 61), (62, 62), (61, 62), (0, w - 1), (h - 1, w - 1), (h - 1, 0)):
            grid[src] = 1
            gg = vector_env.GridGraph(grid)
            assert _bitwise(gg.shortest_path_image(src), O.spfa_image(grid, src)), ((h, w), src)
        free = np.argwhere(grid != 0)
        src = (62, 62)
        tgts = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(6)]
        for t, p in zip(tgts, gg.shortest_paths([(src, t) for t in tgts])):
            want = O.grid_shortest_path(grid, src, t)
            if not np.array_equal(np.array(p, dtype=np.int64).reshape(-1, 2), np.array(want, dtype=np.int64).reshape(-1, 2)):
                assert _dp_tie(grid, src, t), ((h, w), src, t)


def test_whole_window_sweeps_fallback(M):
    """Windows beyond GT_MAXT tiles (>= ~3,968^2 cells) keep the whole-window sweeps (gl_sssp_kernel).
    No test-sized window gets there, so the diagnostic ring build (libsimaps_diagring.so, built with
    SIMAPS_GL_TILE=0) runs every large window through them: images bitwise the oracle's, paths equal
    the product library's (same replay on the same fixpoint)."""
    batch, vector_env = M
    import os
    from simaps import _lib
    L = _lib._load(os.path.join(os.path.dirname(_lib.__file__), 'libsimaps_diagring.so'))
    rs = np.random.RandomState(505)
    for name, grid in _big_grids(rs):
        if name not in ('rand40', 'serpentine'):
            continue
        H, W = grid.shape
        free = np.argwhere(grid != 0)
        srcs = free[rs.randint(len(free), size=2)].astype(np.int32)
        g = torch.from_numpy(grid).cuda().unsqueeze(0).expand(2, H, W).contiguous()
        s = torch.from_numpy(srcs).cuda()
        out = torch.empty((2, H, W), dtype=torch.float32, device='cuda')
        _lib.check(L.simaps_sssp_grid(2, H, W, _lib.ptr(g), _lib.ptr(s), _lib.ptr(out), 0, 0, H, W,
                                      _lib.stream_handle(None)), L)
        got = out.cpu().numpy()
        for k in range(2):
            assert _bitwise(got[k], O.spfa_image(grid, tuple(srcs[k]))), (name, k)
        tg = torch.from_numpy(free[rs.randint(len(free), size=2)].astype(np.int32)).cuda()
        ij = torch.empty((2, 512, 2), dtype=torch.int32, device='cuda')
        cnt = torch.empty((2,), dtype=torch.int32, device='cuda')
        _lib.check(L.simaps_grid_path(2, H, W, _lib.ptr(g), _lib.ptr(s), _lib.ptr(tg), 0, 0, H, W, 512, _lib.ptr(ij),
                                      _lib.ptr(cnt), _lib.stream_handle(None)), L)
        ij2, cnt2 = batch.launch_grid_paths(g, s, tg, max_points=512)
        torch.cuda.synchronize()
        assert torch.equal(cnt, cnt2) and all(torch.equal(ij[k, :int(cnt[k])], ij2[k, :int(cnt2[k])]) for k in range(2))


def test_gridgraph_large_walled_corner_source(M):
    """A source on its tile's corner cell whose only way out is the diagonal into the next tile
    (every other neighbour blocked): the source's own 0 must count as a change of that tile's corner,
    or the diagonal tile is never queued (the tiled fixpoint's initial condition)."""
    batch, vector_env = M
    grid = np.ones((130, 130), np.uint8)
    for s, exit_ in (((61, 61), (62, 62)), ((61, 62), (60, 61)), ((62, 61), (63, 60))):
        g = grid.copy()
        for di in (-1, 0, 1):
            for dj in (-1, 0, 1):
                if (di or dj) and (s[0] + di, s[1] + dj) != exit_:
                    g[s[0] + di, s[1] + dj] = 0
        gg = vector_env.GridGraph(g)
        assert gg.large
        img = gg.shortest_path_image(s)
        assert _bitwise(img, O.spfa_image(g, s)), s
        assert (img > 0).sum() > 10000, s


def test_gridgraph_large_window_offset(M):
    """Free cells that start away from the grid's origin (a blocked margin of 7 rows / 11 columns, and
    a blocked grid corner beyond the window): the window (i0, j0, h, w) the drop-in derives is offset,
    and the tiled fixpoint's tiles, halo and source cell follow it -- images and paths equal the oracle's."""
    batch, vector_env = M
    rs = np.random.RandomState(711)
    grid = np.zeros((300, 400), np.uint8)
    grid[7:280, 11:390] = (rs.random_sample((273, 379)) > 0.3).astype(np.uint8)
    gg = vector_env.GridGraph(grid)
    assert gg.large and gg.window[:2] != (0, 0), gg.window
    free = np.argwhere(grid != 0)
    srcs = [tuple(int(x) for x in free[0]), tuple(int(x) for x in free[-1]), (7 + 61, 11 + 62)]
    grid[srcs[2]] = 1
    gg = vector_env.GridGraph(grid)
    imgs = gg.shortest_path_images(srcs).cpu().numpy()
    for s, img in zip(srcs, imgs):
        assert _bitwise(img, O.spfa_image(grid, s)), s
    tgts = [tuple(int(x) for x in free[rs.randint(len(free))]) for _ in range(4)]
    for t, p in zip(tgts, gg.shortest_paths([(srcs[2], t) for t in tgts])):
        want = O.grid_shortest_path(grid, srcs[2], t)
        if not np.array_equal(np.array(p, dtype=np.int64).reshape(-1, 2), np.array(want, dtype=np.int64).reshape(-1, 2)):
            assert _dp_tie(grid, srcs[2], t), t


def _spiral(n, gap):
    """A rectangular spiral corridor (1 cell wide, walls gap - 1 thick) from the corner (0, 0)."""
    g = np.zeros((n, n), np.uint8)
    top, left, bot, right = 0, 0, n - 1, n - 1
    g[0, :] = 1
    while bot - top >= gap and right - left >= gap:
        g[top:bot + 1, right] = 1
        g[bot, left:right + 1] = 1
        g[top + gap:bot + 1, left] = 1
        top += gap
        g[top, left:right - gap + 1] = 1
        left += gap
        right -= gap
        bot -= gap
    return g


def test_gridgraph_large_spiral(M):
    """The tiled fixpoint's worst case: a 300 x 300 spiral corridor with 1-cell walls passes through
    every tile ~31 times each way (~58 processings per tile in the host model; random grids take
    2-3): the image equals the oracle's, with no fault (the processing cap is a bug guard only)."""
    batch, vector_env = M
    g = _spiral(300, 2)
    gg = vector_env.GridGraph(g)
    assert gg.large
    for src in ((0, 0), (150, 150)):
        if g[src]:
            assert _bitwise(gg.shortest_path_image(src), O.spfa_image(g, src)), src
