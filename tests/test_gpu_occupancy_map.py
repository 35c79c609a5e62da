"""GPU tests of the OccupancyMap drop-in (envs.py:2409-2524): the C-ABI entries
simaps_occupancy_scatter / simaps_build_cspace / simaps_snap_sources and simaps.vector_env.OccupancyMap,
bit for bit against what the reference's own OccupancyMap produced for the scene goldens
(tests/golden/make_goldens.py run_agent: om.update(points, seg, obstacle) on the pixel-centre point
cloud of the agent's occupancy grid, then configuration_space, cspace_thin, closest_cspace_indices and
the shortest-path sources / images), and against the path / reward-lookup goldens."""
import numpy as np
import pytest
import torch

import goldens as G

pytestmark = pytest.mark.gpu

CASES = list(G.scene_cases())


@pytest.fixture(scope='module')
def M():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a GPU (run with -m gpu on an MI355X)')
    from simaps import _lib, batch, constants, synthetic, vector_env
    return _lib, batch, constants, synthetic, vector_env


def _cloud(scene, a, synthetic, K):
    """run_agent's point cloud: one point per pixel centre, seg obstacle where the golden grid is occupied."""
    X, Y = synthetic.pixel_center_positions(scene['H'], scene['W'])
    pts = np.stack([X, Y, np.full_like(X, 0.02)], axis=2).astype(np.float32)
    seg = np.where(scene['occupancy'][a] == 1, K.SEG_VALUES['obstacle'], K.SEG_VALUES['floor']).astype(np.float32)
    return pts, seg


@pytest.mark.parametrize('case', range(0, len(CASES), 3))
def test_occupancy_map_update_vs_reference(M, case):
    """update() from the point cloud reproduces the golden occupancy grid, then configuration_space
    (rect + zeros outside), cspace_thin and the WHOLE closest_cspace_indices table equal the reference's;
    the snapped shortest-path sources and the receptacle image (shortest_path_image) too."""
    _lib, batch, K, synthetic, vector_env = M
    cfg, e, a, scene, pre, z = CASES[case]
    om = vector_env.OccupancyMap(scene['robots'][a]['type'], scene['room_length'], scene['room_width'])
    assert om.configuration_space is None and om.closest_cspace_indices is None
    pts, seg = _cloud(scene, a, synthetic, K)
    om.update(pts, seg, K.SEG_VALUES['obstacle'])
    assert np.array_equal(om.occupancy_map, z[pre + 'occupancy'])
    cs = om.configuration_space
    i0, j0, rh, rw = K.room_rect(scene['room_width'], scene['room_length'])
    want = np.zeros_like(cs)
    want[i0:i0 + rh, j0:j0 + rw] = z[pre + 'cspace_rect']
    assert np.array_equal(cs, want)
    assert np.array_equal(om.cspace_thin, z[pre + 'cspace_thin'])
    assert np.array_equal(om.closest_cspace_indices, z[pre + 'closest'])
    for name in ('receptacle', 'robot'):
        if pre + 'src_' + name not in z.files:
            continue
        pi, pj, si, sj = (int(v) for v in z[pre + 'src_' + name])
        assert tuple(int(v) for v in om._closest_valid_cspace_indices(pi, pj)) == (si, sj)
    if pre + 'sp_receptacle_rect' in z.files:
        img = om.shortest_path_image(scene['receptacle_position'])
        assert img.dtype == np.float32
        want = z[pre + 'sp_receptacle_rect'] / np.float32(96)
        assert np.array_equal(img[i0:i0 + rh, j0:j0 + rw].view(np.int32), want.view(np.int32))
    _lib.check_faults()


def test_build_cspace_and_snap_batched(M):
    """StateBatch.build_cspace / snap_pixels over every agent of a batch in one launch each (and a
    map-slot subset) equal the per-agent golden tables; pixels outside the grid snap to (-1, -1)."""
    _lib, batch, K, synthetic, vector_env = M
    picks = [c for c in CASES if c[0] in ('lifting_4-small_divider', 'lifting_4-large_doors')]
    for cfg, e, a, scene, pre, z in picks:
        b = batch.StateBatch([scene], agents=[(0, a)])
        cs, th = b.build_cspace()
        H, W = scene['H'], scene['W']
        i0, j0, rh, rw = K.room_rect(scene['room_width'], scene['room_length'])
        assert np.array_equal(cs[0].cpu().numpy()[i0:i0 + rh, j0:j0 + rw], z[pre + 'cspace_rect'])
        assert np.array_equal(th[0].cpu().numpy(), z[pre + 'cspace_thin'])
        rs = np.random.RandomState(a)
        px = np.stack([rs.randint(-3, H + 3, 700), rs.randint(-3, W + 3, 700)], -1).astype(np.int32)
        got = b.snap_pixels(px[None]).cpu().numpy()[0]
        inside = (px[:, 0] >= 0) & (px[:, 0] < H) & (px[:, 1] >= 0) & (px[:, 1] < W)
        closest = z[pre + 'closest']
        assert np.array_equal(got[inside], closest[:, px[inside, 0], px[inside, 1]].T)
        assert (got[~inside] == -1).all() and (~inside).sum() > 10
    # a multi-agent batch: one launch for all, a subset by map slots
    cfg, e, a, scene, pre, z = picks[0]
    agents = [(0, k) for k in range(len(scene['robots']))]
    b = batch.StateBatch([scene], agents=agents)
    cs, _ = b.build_cspace(thin=False)
    sub, _ = b.build_cspace(slots=[a], thin=False)
    assert np.array_equal(cs[a].cpu().numpy(), sub[0].cpu().numpy())
    _lib.check_faults()


def test_occupancy_map_paths_and_distances_vs_reference(M):
    """OccupancyMap.shortest_path / shortest_path_distance on the grids of the path and reward-lookup
    goldens (paths.npz: envs 60 + e; sp_distance.npz: envs 40 + e), set through the occupancy_map
    setter: the reference's waypoints (with the caller's own end objects) and distances, exactly."""
    _lib, batch, K, synthetic, vector_env = M
    z = G.load('paths.npz')
    n = 0
    for k in sorted(z.files):
        if not k.endswith('_path') or k.startswith('demo'):
            continue
        key = k[:-len('_path')]
        head, q = key.rsplit('_q', 1)
        cfg, rest = head.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        if int(q) > 1:
            continue
        scene = synthetic.make_scene(cfg, 60 + e)
        om = vector_env.OccupancyMap(scene['robots'][a]['type'], scene['room_length'], scene['room_width'])
        om.occupancy_map = scene['occupancy'][a]
        s, t = tuple(z[key + '_src'].tolist()), tuple(z[key + '_tgt'].tolist())
        p = om.shortest_path(s, t)
        assert p[0] is s and p[-1] is t
        assert np.array_equal(np.array([w[:2] for w in p]), z[key + '_path']), key
        n += 1
    assert n >= 40
    zd = G.load('sp_distance.npz')
    m = 0
    for k in sorted(zd.files):
        if not k.endswith('_dist'):
            continue
        key = k[:-len('_dist')]
        cfg, rest = key.rsplit('_e', 1)
        e, a = (int(x) for x in rest.split('_a'))
        scene = synthetic.make_scene(cfg, 40 + e)
        om = vector_env.OccupancyMap(scene['robots'][a]['type'], scene['room_length'], scene['room_width'])
        om.occupancy_map = scene['occupancy'][a]
        src = zd[key + '_src']
        for t, want in list(zip(zd[key + '_queries'], zd[key + '_dist']))[:4]:
            assert om.shortest_path_distance(src, t) == want, key
            m += 1
    assert m >= 40
    _lib.check_faults()


class LiftingRobot:  # a stand-in of the reference's class (simaps.reference_adapter matches by class name)
    waypoint_positions = [(0.1, -0.05, 0.0), (0.2, 0.1, 0.0), (0.35, 0.12, 0.0)]
    target_end_effector_position = (0.36, 0.14, 0.0)


def _reference_figure(occ, free, fig_w, fig_h, robot, path):
    """OccupancyMap._update_map_visualization + save_figure (envs.py:2529-2555, 2519-2521), restated
    on a pyplot figure (Agg) from the maps the test expects."""
    import matplotlib
    matplotlib.use('Agg')
    import matplotlib.pyplot as plt
    fig = plt.figure(figsize=(4 * fig_w, 4 * fig_h))
    vis = np.zeros(occ.shape) + 0.5
    vis[free == 1] = 1
    vis[occ == 1] = 0
    fig.clf()
    fig.add_axes((0, 0, 1, 1))
    ax = fig.gca()
    ax.axis('off')
    ax.axis([-fig_w / 2, fig_w / 2, -fig_h / 2, fig_h / 2])
    h, w = vis.shape[0] / 96.0, vis.shape[1] / 96.0
    ax.imshow(255.0 * vis, extent=(-w / 2, w / 2, -h / 2, h / 2), cmap='gray', vmin=0, vmax=255.0)
    wp = np.array(robot.waypoint_positions)
    ax.plot(wp[:, 0], wp[:, 1], color='r', marker='.')
    ax.plot(robot.target_end_effector_position[0], robot.target_end_effector_position[1], color='r', marker='x')
    fig.savefig(path, bbox_inches='tight', pad_inches=0)
    plt.close(fig)


def test_occupancy_map_show_map_figure(M, tmp_path):
    """show_map=True: the free-space map (envs.py:2462-2465: every point whose seg is not np.isclose to
    the obstacle value, NaN included) equals the host rule's, over two updates; save_figure's PNG equals
    the reference's drawing steps on the expected maps, pixel for pixel."""
    from PIL import Image
    _lib, batch, K, synthetic, vector_env = M
    cfg, e, a, scene, pre, z = CASES[0]
    robot = LiftingRobot()
    om = vector_env.OccupancyMap(robot, scene['room_length'], scene['room_width'], show_map=True)
    assert not om.free_space_map.any()
    pts, seg = _cloud(scene, a, synthetic, K)
    rs = np.random.RandomState(7)
    # a sparse first frame: a third of the points, some segs NaN or a hair off the obstacle value
    keep = rs.rand(*seg.shape) < 0.35
    seg1 = np.where(keep, seg, np.float32(K.SEG_VALUES['floor'])).astype(np.float32)
    seg1[rs.rand(*seg.shape) < 0.01] = np.nan
    ob = np.float32(K.SEG_VALUES['obstacle'])
    seg1[rs.rand(*seg.shape) < 0.01] = ob * np.float32(1 + 4e-6)
    pts1 = np.where(keep[..., None], pts, np.float32(9.0))  # dropped points land clipped at the border
    free = np.zeros((scene['H'], scene['W']), np.uint8)
    occ = np.zeros_like(free)
    for p, s in ((pts1, seg1), (pts, seg)):
        om.update(p, s, K.SEG_VALUES['obstacle'])
        close = np.isclose(s, K.SEG_VALUES['obstacle']).reshape(-1)
        px, py = p.reshape(-1, 3)[:, 0], p.reshape(-1, 3)[:, 1]  # position_to_pixel_indices on float32
        pi = np.clip(np.floor(free.shape[0] / 2 - py * 96.0).astype(np.int32), 0, free.shape[0] - 1)
        pj = np.clip(np.floor(free.shape[1] / 2 + px * 96.0).astype(np.int32), 0, free.shape[1] - 1)
        free[pi[~close], pj[~close]] = 1
        occ[pi[close], pj[close]] = 1
        assert np.array_equal(om.free_space_map, free)
        assert np.array_equal(om.occupancy_map, occ)
    assert occ.sum() > 100 and free.sum() > 1000
    om.save_figure(tmp_path / 'global-occupancy-map.png')
    _reference_figure(occ, free, om.fig_width, om.fig_height, robot, tmp_path / 'want.png')
    got = np.asarray(Image.open(tmp_path / 'global-occupancy-map.png'))
    want = np.asarray(Image.open(tmp_path / 'want.png'))
    assert got.shape == want.shape and got.shape[0] > 100
    assert np.array_equal(got, want)
    _lib.check_faults()
