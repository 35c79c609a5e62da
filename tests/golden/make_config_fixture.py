"""Fixture generator (run in the dev container, where /root/reference exists): the state-
representation flags, room, robots and num_input_channels of every reference experiment config
(config/**/*.yml, yaml.safe_load), with VectorEnv.__init__'s defaults for the three flags a config
may omit (envs.py:37-45; utils.get_env_from_cfg, utils.py:182-195 allows exactly those), and the
overrides train.py applies when it builds the env of a predicted-intention config (train.py:172-174:
the ground-truth intention map, ramp encoding, is on during training).  Output:
tests/golden/reference_configs.json (data only)."""
import glob
import json
import os

import yaml

REF = '/root/reference/config'
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'reference_configs.json')
KEYS = ['use_robot_map', 'use_distance_to_receptacle_map', 'distance_to_receptacle_map_scale',
        'use_shortest_path_to_receptacle_map', 'use_shortest_path_map', 'shortest_path_map_scale',
        'use_intention_map', 'intention_map_encoding', 'intention_map_scale', 'intention_map_line_thickness',
        'use_history_map', 'use_intention_channels', 'intention_channel_encoding',
        'intention_channel_nonspatial_scale']
DEFAULTS = {'use_robot_map': True, 'intention_map_scale': 1.0, 'intention_map_line_thickness': 2}  # envs.py:40-42


def main():
    rows = []
    for path in sorted(glob.glob(os.path.join(REF, '**', '*.yml'), recursive=True)):
        cfg = yaml.safe_load(open(path))
        flags = {k: cfg.get(k, DEFAULTS.get(k)) for k in KEYS}
        if cfg.get('use_predicted_intention'):  # train.py:172-174
            flags.update(use_intention_map=True, intention_map_encoding='ramp')
        missing = [k for k in KEYS if flags[k] is None]
        assert not missing, (path, missing)
        rows.append({'config': os.path.relpath(path, REF), 'flags': flags, 'room_length': cfg['room_length'],
                     'room_width': cfg['room_width'], 'env_name': cfg['env_name'],
                     'robot_config': cfg['robot_config'], 'num_input_channels': cfg['num_input_channels'],
                     'use_predicted_intention': bool(cfg.get('use_predicted_intention'))})
    json.dump(rows, open(OUT, 'w'), indent=0, sort_keys=True)
    print(len(rows), 'configs ->', OUT)


if __name__ == '__main__':
    main()
