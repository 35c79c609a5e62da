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
