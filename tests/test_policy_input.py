"""CPU: policy input -- apply_transform keeps ToTensor semantics for
NumPy states and is a zero-copy view for CHW-rendered states."""
import numpy as np
import pytest
import torch

from simaps import policy_input


def test_apply_transform_numpy_matches_totensor_semantics():
    s = np.random.RandomState(0).rand(96, 96, 5).astype(np.float32)
    t = policy_input.apply_transform(s)
    assert tuple(t.shape) == (1, 5, 96, 96) and t.dtype == torch.float32
    assert np.array_equal(t[0].numpy(), s.transpose(2, 0, 1))       # float input: no scaling


def test_apply_transform_chw_view_is_zero_copy():
    chw = torch.rand(4, 5, 96, 96)
    hwc = chw.permute(0, 2, 3, 1)                                     # StateBatch.as_hwc view
    t = policy_input.apply_transform(hwc[2])
    assert t.data_ptr() == chw[2].data_ptr() and torch.equal(t[0], chw[2])
    batches = policy_input.group_batches([[hwc[0], None], [hwc[3], hwc[1]]])
    assert batches[0][0] == [0] and torch.equal(batches[0][1], chw[0:1])
    assert batches[1][0] == [0, 1] and torch.equal(batches[1][1], torch.stack([chw[3], chw[1]]))


def test_intention_policy_channel_transforms():
    """DQNIntentionPolicy's state edits (policies.py:97-108, 126-131) on CHW batches equal the
    reference's HWC NumPy edits followed by apply_transform."""
    rs = np.random.RandomState(3)
    states = [rs.rand(96, 96, 5).astype(np.float32) for _ in range(3)]
    preds = [rs.rand(96, 96).astype(np.float32) for _ in range(3)]
    batch = torch.cat([policy_input.apply_transform(s) for s in states])
    dropped = policy_input.without_intention_map(batch)
    assert dropped.data_ptr() == batch.data_ptr()  # a view, no copy
    ref = torch.cat([policy_input.apply_transform(np.ascontiguousarray(s[:, :, :-1])) for s in states])
    assert torch.equal(dropped, ref)
    got = policy_input.with_predicted_intention(dropped, torch.from_numpy(np.stack(preds)))
    ref = torch.cat([policy_input.apply_transform(np.concatenate((s[:, :, :-1], np.expand_dims(o, 2)), axis=2))
                     for s, o in zip(states, preds)])
    assert got.shape == (3, 5, 96, 96) and torch.equal(got, ref)
    with pytest.raises(ValueError):
        policy_input.with_predicted_intention(dropped, torch.zeros(2, 96, 96))
