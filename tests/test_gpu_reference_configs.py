"""GPU: one scene pair for every one of the reference's 93 experiment configs (config/**/*.yml, as
tests/golden/reference_configs.json holds them: env_name, robots, state-representation flags),
every agent rendered through the C ABI and checked against the oracle at the bar of
test_gpu_parity.py; the rotate rounding alternates between configs."""
import json
import os

import pytest
import torch

import oracle as O
from test_gpu_parity import _check_state

pytestmark = pytest.mark.gpu

ROWS = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'reference_configs.json')))


@pytest.fixture(scope='module')
def S():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a GPU (run with -m gpu on an MI355X)')
    from simaps import batch, synthetic
    return batch, synthetic


@pytest.mark.parametrize('k', range(len(ROWS)), ids=[r['config'] for r in ROWS])
def test_reference_config_vs_oracle(S, k):
    batch, synthetic = S
    row = ROWS[k]
    rounding = 'plain' if k % 2 else 'fma'
    scenes = [dict(synthetic.reference_config_scene(row, 10 * k + e), rotate_rounding=rounding) for e in range(2)]
    b = batch.StateBatch(scenes, layout='hwc' if k % 3 else 'chw')
    assert b.C == row['num_input_channels']
    st = b.as_hwc(b.render()).cpu().numpy()
    for n, (e, a) in enumerate(b.agents):
        _check_state(st[n], O.agent_state(scenes[e], a), scenes[e]['flags'], len(scenes[e]['robots']))


@pytest.mark.parametrize('k', range(len(ROWS)), ids=[r['config'] for r in ROWS])
def test_reference_config_rows_vs_oracle(S, k):
    """The 8(f) rows on each reference config's scene (fully observed maps: long detours): every
    agent's movement path to 3 targets across the room (OccupancyMap.shortest_path) and its reward
    lookups (shortest_path_distance) against the oracle; a path may differ only at an
    approximate_polygon floating-point tie (test_gpu_dropin.py)."""
    import numpy as np
    from test_gpu_dropin import _dp_tie
    batch, synthetic = S
    row = ROWS[k]
    s = synthetic.reference_config_scene(row, 1000 + k, observe_all=True)
    b = batch.StateBatch([s])
    rs = np.random.RandomState(k)
    rl, rw = s['room_length'], s['room_width']
    src = np.array([s['robots'][a]['position'][:2] for _, a in b.agents])
    tgt = np.stack([rs.uniform(-rl / 2 + 0.02, rl / 2 - 0.02, (b.N, 3)), rs.uniform(-rw / 2 + 0.02, rw / 2 - 0.02, (b.N, 3))], -1)
    paths = [b.shortest_paths(src, tgt[:, q]) for q in range(3)]
    d = b.shortest_path_distances(src, tgt).cpu().numpy()
    ties = 0
    for n, (_, a) in enumerate(b.agents):
        ao = O.AgentOracle(s, a)
        for q in range(3):
            assert d[n, q] == ao.shortest_path_distance(src[n], tgt[n, q]), (n, q)
            want = np.array(ao.shortest_path(src[n], tgt[n, q]), dtype=np.float64).reshape(-1, 2)
            got = np.array([p[:2] for p in paths[q][n]], dtype=np.float64).reshape(-1, 2)
            if not np.array_equal(got, want):
                assert _dp_tie(ao.cspace, ao.snap(src[n]), ao.snap(tgt[n, q])), (n, q)
                ties += 1
    assert ties <= 1
