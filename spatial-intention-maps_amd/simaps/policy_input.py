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


def without_intention_map(batch):
    """DQNIntentionPolicy.step in training (policies.py:126-131): the ground-truth intention map,
    the state's last channel, removed before the intention network runs -- s[:, :, :-1] on a
    (96, 96, C) state; here a zero-copy view of an [n, C, 96, 96] batch (its first C - 1 planes)."""
    if batch.dim() != 4:
        raise ValueError('expected an [n, C, 96, 96] batch')
    return batch[:, :-1]


def with_predicted_intention(batch, intention):
    """DQNIntentionPolicy.step_intention (policies.py:97-108): the intention network's sigmoid
    output appended as the last channel -- np.concatenate((s, o[:, :, None]), axis=2) on a
    (96, 96, C) state; here [n, C, 96, 96] + [n, 96, 96] (or [n, 1, 96, 96]) -> [n, C + 1, 96, 96]."""
    if intention.dim() == 3:
        intention = intention.unsqueeze(1)
    if batch.dim() != 4 or intention.shape != (batch.shape[0], 1) + tuple(batch.shape[2:]):
        raise ValueError('expected [n, C, H, W] states and [n, H, W] intention maps')
    return torch.cat([batch, intention.to(batch.dtype)], 1)
