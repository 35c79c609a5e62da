"""CPU: policy input -- apply_transform keeps ToTensor semantics for
NumPy states and is a zero-copy view for CHW-rendered states."""
import numpy as np
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
