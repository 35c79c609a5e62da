"""Policy input from device-resident stacks.

The reference feeds each awaiting robot's state to its group's network one at a time
(DQNPolicy.step, policies.py:49-66) through apply_transform (policies.py:44-45):
torchvision ToTensor on a (96, 96, C) float32 NumPy array = the (C, 96, 96) tensor (float input:
no scaling), unsqueezed to a batch of one, then copied host -> device.

Stacks rendered by simaps stay on the GPU in the CHW layout the networks consume, so the
equivalent is a view (no copy, no transpose), and a whole robot group can go through its network
in one batch.
"""
import numpy as np
import torch


def apply_transform(s, device=None):
    """DQNPolicy.apply_transform for either a reference state ((96, 96, C) NumPy float32) or a
    simaps state (a (96, 96, C) view of a CHW device tensor): -> [1, C, 96, 96] float32."""
    if isinstance(s, np.ndarray):
        if s.dtype != np.float32 or s.ndim != 3:
            raise ValueError('expected a (H, W, C) float32 state')
        t = torch.from_numpy(np.ascontiguousarray(s.transpose(2, 0, 1)))  # ToTensor: HWC -> CHW
        return t.unsqueeze(0) if device is None else t.unsqueeze(0).to(device)
    t = s.permute(2, 0, 1)  # the HWC view of a CHW tensor -> the CHW tensor itself
    return t.unsqueeze(0) if device is None else t.unsqueeze(0).to(device)


def group_batches(state):
    """One env's VectorEnv.get_state structure ([group][robot] -> state or None) -> per group
    (robot indices, [n, C, 96, 96] batch) for one network call per group instead of per robot."""
    out = []
    for g in state:
        idx = [j for j, s in enumerate(g) if s is not None]
        out.append((idx, torch.cat([apply_transform(g[j]) for j in idx]) if idx else None))
    return out
