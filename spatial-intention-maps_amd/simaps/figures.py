"""Mapper.get_state(save_figures=True)'s map PNGs (envs.py:2115-2182), host side.

The reference writes, per robot, into figures/robot_id_<id>/: the simulator camera image (env.png),
the global and local overhead maps, and for every map channel its global and local maps blended over
the overhead map through the jet colormap (utils.JET / to_uint8_image / enlarge_image, utils.py:95-98,
153-154), plus the intention channels.  Here the maps come from the device: the local maps are the
rendered state's channels, the global ones simaps_global_maps / StateBatch.shortest_path_images.  Not
written: env.png (a pybullet camera render; there is no simulator here).  global-occupancy-map.png is
OccupancyMap.save_figure (vector_env.OccupancyMap with show_map=True, passed to get_state).  PIL and
matplotlib are needed only by this debug path, as in the reference.
"""
from pathlib import Path

import numpy as np

from . import constants as K

_JET = None


def jet():
    """utils.JET (utils.py:95): matplotlib's 256-entry jet colormap, RGB float32."""
    global _JET
    if _JET is None:
        from matplotlib import cm
        _JET = np.array([list(cm.jet(i)[:3]) for i in range(256)], dtype=np.float32)
    return _JET


def to_uint8_image(image):
    """utils.to_uint8_image (utils.py:97-98)."""
    return np.round(255.0 * image).astype(np.uint8)


def enlarge_image(image, scale_factor=4):
    """utils.enlarge_image (utils.py:153-154): PIL nearest-neighbour resize."""
    from PIL import Image
    return image.resize((scale_factor * image.size[0], scale_factor * image.size[1]), resample=Image.NEAREST)


def _save(arr, path):
    from PIL import Image
    enlarge_image(Image.fromarray(to_uint8_image(arr))).save(path)


def global_map_room_only(global_map, room_length, room_width):
    """get_state's global_map_room_only (envs.py:2122-2127)."""
    crop_width = K.round_up_to_even((room_length + 2 * K.HALF_WIDTH) * K.LOCAL_MAP_PIXELS_PER_METER)
    crop_height = K.round_up_to_even((room_width + 2 * K.HALF_WIDTH) * K.LOCAL_MAP_PIXELS_PER_METER)
    start_i = global_map.shape[0] // 2 - crop_height // 2
    start_j = global_map.shape[1] // 2 - crop_width // 2
    return global_map[start_i:start_i + crop_height, start_j:start_j + crop_width]


def channel_names(flags, num_robots):
    """The state's channels in envs.py:2071-2113 order: (name, figure suffix or None)."""
    names = [('overhead', None)]
    if flags['use_robot_map']:
        names.append(('robot', 'robot-map'))
    if flags['use_distance_to_receptacle_map']:
        names.append(('distance_to_receptacle', None))  # (no figure in the reference)
    if flags['use_shortest_path_to_receptacle_map']:
        names.append(('sp_receptacle', 'shortest-path-to-receptacle-map'))
    if flags['use_shortest_path_map']:
        names.append(('sp_robot', 'shortest-path-map'))
    if flags['use_history_map']:
        names.append(('history', 'history-map'))
    if flags['use_intention_map']:
        names.append(('intention', 'intention-map'))
    if flags['use_intention_channels']:
        per = 1 if flags['intention_channel_encoding'] == 'spatial' else 2
        names += [('intention_channel%d' % i, None) for i in range(per * (num_robots - 1))]
    return names


def save_state_figures(output_dir, flags, room_length, room_width, num_robots, state, global_maps):
    """Write get_state's PNGs for one robot into output_dir (created if missing).

    state: its (96, 96, C) float32 state (the local maps); global_maps: the whole-grid maps by channel
    name ('overhead', and 'robot' / 'sp_receptacle' / 'sp_robot' / 'history' / 'intention' as the flags
    enable them), float32 NumPy.  Returns the list of files written."""
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    names = channel_names(flags, num_robots)
    local = {name: state[:, :, c] for c, (name, _) in enumerate(names)}
    written = []

    def save(arr, name):
        _save(arr, out / name)
        written.append(out / name)

    room = lambda m: global_map_room_only(m, room_length, room_width)  # noqa: E731
    brightness_scale_factor = 1.33  # visualize_overhead_map (envs.py:2132-2136)
    global_overhead_map_vis = brightness_scale_factor * room(global_maps['overhead'])
    local_overhead_map_vis = brightness_scale_factor * local['overhead']
    save(global_overhead_map_vis, 'global-overhead-map.png')
    save(local_overhead_map_vis, 'local-overhead-map.png')

    def visualize_map(overhead_map_vis, distance_map):  # envs.py:2143-2146
        overhead_map_vis = np.stack(3 * [overhead_map_vis], axis=2)
        distance_map_vis = jet()[to_uint8_image(distance_map), :]
        return 0.5 * overhead_map_vis + 0.5 * distance_map_vis

    def save_map_visualization(global_map, local_map, suffix, scale=1):  # envs.py:2148-2153
        save(visualize_map(global_overhead_map_vis, scale * room(global_map)), 'global-{}.png'.format(suffix))
        save(visualize_map(local_overhead_map_vis, scale * local_map), 'local-{}.png'.format(suffix))

    for name, suffix in names:
        if suffix is None:
            continue
        scale = 2 if name.startswith('sp_') else 1
        save_map_visualization(global_maps[name], local[name], suffix, scale)
    k = 0
    for name, _ in names:
        if name.startswith('intention_channel'):
            save(visualize_map(local_overhead_map_vis, np.abs(local[name])), 'intention-channel{}.png'.format(k))
            k += 1
    return written


def device_global_maps(b, slots, positions):
    """The global maps save_state_figures needs, for map slots `slots` of StateBatch b: the
    simaps_global_maps outputs, and the shortest-path maps of _create_global_shortest_path_to_receptacle_map
    / _create_global_shortest_path_map (envs.py:2287-2300: shortest_path_image, unreachable -> its max,
    x shortest_path_map_scale) from the device images.  positions: each slot's robot (x, y).  Returns
    one dict of float32 NumPy arrays per slot."""
    g = {k: v.cpu().numpy() for k, v in b.global_maps(slots=slots).items()}
    flags = b.flags
    scale = np.float32(flags['shortest_path_map_scale'])

    def sp(img):
        img = img.copy()
        img[img < 0] = img.max()
        img *= scale
        return img
    if flags['use_shortest_path_to_receptacle_map']:
        rec = np.array([b.scenes[b.agents[k][0]]['receptacle_position'][:2] for k in slots], dtype=np.float64)
        g['sp_receptacle'] = np.stack([sp(m) for m in b.shortest_path_images(rec, slots=slots).cpu().numpy()])
    if flags['use_shortest_path_map']:
        g['sp_robot'] = np.stack([sp(m) for m in b.shortest_path_images(np.asarray(positions, dtype=np.float64), slots=slots)
                                  .cpu().numpy()])
    return [{k: v[i] for k, v in g.items()} for i in range(len(slots))]
