"""Loaders for the committed golden fixtures (tests/golden/*.npz, made by make_goldens.py)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def scene_files():
    return sorted(glob.glob(os.path.join(GOLDEN, 'scene_*.npz')))


def scene_cases():
    """Yield (config, env_idx, agent, scene_dict, arrays_prefix, npz) for every golden agent."""
    for path in scene_files():
        z = np.load(path, allow_pickle=False)
        e = 0
        while 'e%d_scene' % e in z.files:
            scene = json.loads(str(z['e%d_scene' % e]))
            if 'rotate_rounding' not in scene:  # (make_goldens.py records the rendering host's rounding)
                raise ValueError('%s e%d: scene descriptor without rotate_rounding' % (os.path.basename(path), e))
            # (robots that have not acted yet carry None paths / target: the reset goldens)
            scene['robots'] = [dict(r, position=tuple(r['position']),
                                    target_ee=None if r['target_ee'] is None else tuple(r['target_ee']),
                                    waypoint_positions=None if r['waypoint_positions'] is None else
                                    [tuple(p) for p in r['waypoint_positions']])
                               for r in scene['robots']]
            if scene['receptacle_position'] is not None:
                scene['receptacle_position'] = tuple(scene['receptacle_position'])
            agents = z['e%d_agents' % e]
            A = len(scene['robots'])
            H, W = scene['H'], scene['W']
            occ = np.zeros((A, H, W), np.uint8)
            ovh = np.zeros((A, H, W), np.float32)
            for a in agents:
                occ[a] = z['e%d_a%d_occupancy' % (e, a)]
                ovh[a] = z['e%d_a%d_overhead' % (e, a)]
            scene['occupancy'], scene['overhead'] = occ, ovh
            for a in agents:
                yield scene['config'], e, int(a), scene, 'e%d_a%d_' % (e, a), z
            e += 1
