"""GPU: one launch over envs of several configurations (simaps_get_state_mixed, MixedStateBatch)
against one StateBatch render per configuration and against the oracle.  The bar is the one of
test_gpu_parity.py: bit-exact, except the nonspatial intention channels (1e-7 absolute vs the
oracle; bit-exact vs the per-configuration kernel, which runs the same device code)."""
import numpy as np
import pytest
import torch

import oracle as O
from test_gpu_parity import _bitwise, _check_state

pytestmark = pytest.mark.gpu

# 8 configurations (the most one launch takes): both grid sizes, every channel family, both host
# roundings of rotate's out_center; env counts ragged per configuration
MIX = [('lifting_4-small_divider', 'fma', 3), ('pushing_4-large_empty', 'fma', 2), ('rescue_4-small_empty', 'fma', 1),
       ('lifting_4-small_divider-history', 'plain', 2), ('lifting_4-large_empty-line', 'fma', 1),
       ('lifting_4-small_divider-spatial', 'fma', 2), ('lifting_4-large_empty-nonspatial', 'plain', 2),
       ('lifting_2_pushing_2-large_empty-all', 'fma', 1)]


@pytest.fixture(scope='module')
def S():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a GPU (run with -m gpu on an MI355X)')
    from simaps import _lib, batch, synthetic
    return _lib, batch, synthetic


def _mixed_scenes(synthetic, seed=300):
    """Configurations interleaved env by env (not grouped), so slots of one configuration are not
    contiguous in the launch."""
    per = [[dict(synthetic.make_scene(c, seed + 10 * k + e), rotate_rounding=r) for e in range(n)]
           for k, (c, r, n) in enumerate(MIX)]
    out = []
    while any(per):
        for p in per:
            if p:
                out.append(p.pop(0))
    return out


def _per_config_stacks(batch, scenes, layout):
    """{(env, robot): stack} from one StateBatch render per configuration."""
    groups = {}
    for e, s in enumerate(scenes):
        groups.setdefault(batch.config_key(s), []).append(e)
    got = {}
    for envs in groups.values():
        b = batch.StateBatch([scenes[e] for e in envs], layout=layout)
        st = b.render().cpu().numpy()
        for n, (i, a) in enumerate(b.agents):
            got[(envs[i], a)] = st[n]
    return got


@pytest.mark.parametrize('layout', ['chw', 'hwc'])
def test_mixed_equals_per_configuration_renders(S, layout):
    _lib, batch, synthetic = S
    scenes = _mixed_scenes(synthetic)
    mb = batch.MixedStateBatch(scenes, layout=layout)
    assert len(mb.plan['cfgs']) == 8
    out = mb.render()
    views = [v.cpu().numpy() for v in mb.states(out)]
    _lib.check_faults()
    ref = _per_config_stacks(batch, scenes, layout)
    for n, (e, a) in enumerate(mb.agents):
        assert _bitwise(views[n], ref[(e, a)]), (n, e, a)


def test_mixed_vs_oracle(S):
    _lib, batch, synthetic = S
    scenes = _mixed_scenes(synthetic, seed=400)
    mb = batch.MixedStateBatch(scenes, layout='hwc')
    views = [v.cpu().numpy() for v in mb.states(mb.render())]
    _lib.check_faults()
    for n, (e, a) in enumerate(mb.agents):
        _check_state(views[n], O.agent_state(scenes[e], a), scenes[e]['flags'], len(scenes[e]['robots']))


def test_mixed_full_size_single_and_two_configs(S):
    """A benchmark-sized launch: 64 envs of lifting_4-small_divider alone (mixed == StateBatch) and
    beside 64 of pushing_4-large_empty; deterministic across renders and streams."""
    _lib, batch, synthetic = S
    a = [synthetic.make_scene('lifting_4-small_divider', 500 + e) for e in range(64)]
    b = [synthetic.make_scene('pushing_4-large_empty', 600 + e) for e in range(64)]
    sb = batch.StateBatch(a)
    ref_a = sb.render().cpu().numpy()
    mb = batch.MixedStateBatch(a)
    got = mb.render().view(len(sb.agents), sb.C, 96, 96).cpu().numpy()
    assert _bitwise(got, ref_a)
    mb2 = batch.MixedStateBatch(a + b)
    side = torch.cuda.Stream()
    o1 = mb2.render()
    o2 = mb2.render(stream=side)
    torch.cuda.current_stream().wait_stream(side)
    v1, v2 = o1.cpu().numpy(), o2.cpu().numpy()
    assert _bitwise(v1, v2)
    ref_b = batch.StateBatch(b).render().cpu().numpy()
    na = len(sb.agents)
    assert _bitwise(v1[:ref_a.size].reshape(ref_a.shape), ref_a)
    assert _bitwise(v1[ref_a.size:].reshape(ref_b.shape), ref_b)
    assert len(mb2.agents) == na + 4 * 64
    _lib.check_faults()


def test_mixed_graph_capture_replays(S):
    """The mixed launch allocates nothing: it captures into a graph, and a replay after new
    descriptors were copied into the captured buffers renders the new scenes."""
    _lib, batch, synthetic = S
    s1 = _mixed_scenes(synthetic, seed=700)
    s2 = _mixed_scenes(synthetic, seed=800)
    mb = batch.MixedStateBatch(s1)
    p1, p2 = (np.ascontiguousarray(batch.pack_descriptors(s, mb.agents)[3]).view(np.uint8).reshape(-1) for s in (s1, s2))
    mb.paths_d = torch.zeros(max(p1.size, p2.size), dtype=torch.uint8, device=mb.device)  # room for both
    mb.paths_d[:p1.size].copy_(torch.from_numpy(p1))
    out = mb.alloc_state()
    mb.render(out)  # warm-up outside the capture
    torch.cuda.synchronize()
    bufs = (mb.robots_d, mb.envs_d, mb.agents_d, mb.paths_d)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        mb.render(out)
    # the second scenes' descriptors, copied into the captured buffers (same robot counts per env,
    # so the same agents and descriptor sizes; the path buffer has room for either)
    for dst, src in zip(bufs, batch.pack_descriptors(s2, mb.agents)):
        src = torch.from_numpy(np.ascontiguousarray(src).view(np.uint8).reshape(-1))
        assert src.numel() <= dst.numel()
        dst[:src.numel()].copy_(src)
    occ = np.concatenate([np.asarray(s2[e]['occupancy'][a], dtype=np.uint8).ravel() for e, a in mb.agents])
    ovh = np.concatenate([np.asarray(s2[e]['overhead'][a], dtype=np.float32).ravel() for e, a in mb.agents])
    mb.occupancy.copy_(torch.from_numpy(occ))
    mb.overhead.copy_(torch.from_numpy(ovh))
    g.replay()
    got = [v.cpu().numpy() for v in mb.states(out)]
    _lib.check_faults()
    ref = _per_config_stacks(batch, s2, 'chw')
    for n, (e, a) in enumerate(mb.agents):
        assert _bitwise(got[n], ref[(e, a)]), n


def test_mixed_bad_configuration_index_is_reported(S):
    _lib, batch, synthetic = S
    scenes = _mixed_scenes(synthetic, seed=900)
    mb = batch.MixedStateBatch(scenes)
    clean = [v.cpu().numpy() for v in mb.states(mb.render())]
    _lib.check_faults()
    # agent 0's configuration index past the table: the fault is reported and its workgroup writes
    # nothing (no configuration's channel count is known to fit its stack); every other agent renders
    mb.agent_cfg_d[0] = 99
    out = mb.alloc_state().fill_(float("nan"))
    torch.cuda.synchronize()
    got = [v.cpu().numpy() for v in mb.states(mb.render(out=out))]
    with pytest.raises(_lib.DeviceFault, match='descriptor-clamped'):
        _lib.check_faults()
    assert np.isnan(got[0]).all()
    for n in range(1, mb.N):
        assert _bitwise(got[n], clean[n]), n


@pytest.mark.parametrize('count', [3, 5])
def test_intention_channel_robot_count_mismatch_is_contained(S, count):
    """An env whose robot count differs from the one the intention channels were sized for (the
    C ABI cannot check device descriptors) is clamped and reported; it never writes past its own
    stacks, so the other envs' agents render as before -- both entry points."""
    _lib, batch, synthetic = S
    scenes = [synthetic.make_scene('lifting_4-large_empty-nonspatial', 950 + e) for e in range(3)]
    for make in (lambda: batch.StateBatch(scenes), lambda: batch.MixedStateBatch(scenes)):
        b = make()
        clean = b.render().cpu().numpy().reshape(12, -1)
        _lib.check_faults()
        b.envs_d.view(torch.int32)[6] = count  # env 0's num_robots (simaps_env: byte offset 24)
        torch.cuda.synchronize()
        got = b.render().cpu().numpy().reshape(12, -1)
        with pytest.raises(_lib.DeviceFault, match='descriptor-clamped'):
            _lib.check_faults()
        assert _bitwise(got[4:], clean[4:])


def test_mixed_set_maps(S):
    """set_maps on a subset of slots and on all of them: the render equals one StateBatch per
    configuration over scenes holding the new maps."""
    _lib, batch, synthetic = S
    scenes = _mixed_scenes(synthetic, seed=1100)
    other = _mixed_scenes(synthetic, seed=1200)  # same configurations and robot counts, other maps
    mb = batch.MixedStateBatch(scenes)
    want = [dict(s, occupancy=np.array(s['occupancy']), overhead=np.array(s['overhead'])) for s in scenes]
    slots = [0, 3, 7, 12, mb.N - 1]
    pairs = [mb.agents[k] for k in slots]
    mb.set_maps(occupancy=[other[e]['occupancy'][a] for e, a in pairs],
                overhead=[torch.as_tensor(other[e]['overhead'][a]).cuda() for e, a in pairs], slots=slots)
    for e, a in pairs:
        want[e]['occupancy'][a] = other[e]['occupancy'][a]
        want[e]['overhead'][a] = other[e]['overhead'][a]
    got = [v.cpu().numpy() for v in mb.states(mb.render())]
    ref = _per_config_stacks(batch, want, 'chw')
    for n, (e, a) in enumerate(mb.agents):
        assert _bitwise(got[n], ref[(e, a)]), n
    mb.set_maps(occupancy=[other[e]['occupancy'][a] for e, a in mb.agents],
                overhead=[other[e]['overhead'][a] for e, a in mb.agents])
    got = [v.cpu().numpy() for v in mb.states(mb.render())]
    ref = _per_config_stacks(batch, [dict(s, occupancy=o['occupancy'], overhead=o['overhead'])
                                     for s, o in zip(scenes, other)], 'chw')
    for n, (e, a) in enumerate(mb.agents):
        assert _bitwise(got[n], ref[(e, a)]), n
    _lib.check_faults()
    e, a = mb.agents[0]
    small = np.zeros((3, 3), np.uint8)
    with pytest.raises(ValueError, match='must have shape'):
        mb.set_maps(occupancy=[small], slots=[0])
    with pytest.raises(ValueError, match='one map per slot'):
        mb.set_maps(occupancy=[small, small], slots=[0])


@pytest.mark.parametrize('cfg', ['lifting_4-large_empty-nonspatial', 'lifting_4-small_divider-spatial'])
def test_mixed_intention_channels_ragged_robot_counts(S, cfg):
    """Intention channels with 4-, 3- and 2-robot envs of one configuration: one table entry per
    robot count (their channel counts differ), one launch, each agent as its own StateBatch and the
    oracle render it."""
    _lib, batch, synthetic = S

    def trimmed(e, n):
        s = synthetic.make_scene(cfg, 1300 + e)
        return dict(s, robots=s['robots'][:n], occupancy=s['occupancy'][:n], overhead=s['overhead'][:n])
    scenes = [trimmed(0, 4), trimmed(1, 3), trimmed(2, 2), trimmed(3, 3), trimmed(4, 4)]
    mb = batch.MixedStateBatch(scenes, layout='hwc')
    assert len(mb.plan['cfgs']) == 3
    got = [v.cpu().numpy() for v in mb.states(mb.render())]
    _lib.check_faults()
    for n, (e, a) in enumerate(mb.agents):
        _check_state(got[n], O.agent_state(scenes[e], a), scenes[e]['flags'], len(scenes[e]['robots']))
    for e in range(len(scenes)):
        ref = batch.StateBatch([scenes[e]], layout='hwc').render().cpu().numpy()
        for n, (e2, a) in enumerate(mb.agents):
            if e2 == e:
                assert _bitwise(got[n], ref[a]), (e, a)


def test_mixed_descriptor_arrays_match_scene_update(S):
    """The array fast path (native simaps_pack_robots, one pinned upload) on a mixed batch renders
    what set_descriptors of the same scenes renders."""
    _lib, batch, synthetic = S
    scenes = _mixed_scenes(synthetic, seed=1400)
    moved = _mixed_scenes(synthetic, seed=1500)  # other poses, targets and paths of the same robots
    mb = batch.MixedStateBatch(scenes)
    mb.set_descriptor_arrays(**batch.descriptor_arrays(moved))
    got = mb.render().cpu().numpy()
    mb.set_descriptors([dict(s, robots=m['robots'], receptacle_position=s['receptacle_position'])
                        for s, m in zip(scenes, moved)])
    want = mb.render().cpu().numpy()
    _lib.check_faults()
    assert _bitwise(got, want)
