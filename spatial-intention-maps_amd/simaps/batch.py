"""Device-resident batches of agent-state stacks and the fused get_state launch.

A StateBatch packs E envs x (their agents) of ONE configuration (same grid / flags) into HBM:
  occupancy  u8  [N, H, W]   per-agent OccupancyMap.occupancy_map      (envs.py:2417, 2447-2450)
  overhead   f32 [N, H, W]   per-agent global_overhead_map_without_robots (envs.py:2026, 2057-2062)
  robots / envs / agents / paths: the per-step scene descriptor (poses, controller state, paths)
and renders every agent's (96, 96, C) float32 stack in one kernel launch.  The per-agent maps are
meant to stay resident across steps (the reference keeps them in each robot's Mapper); only the
descriptor (~100 B per robot) changes per step.  A MixedStateBatch renders envs of up to 8
configurations in one launch (simaps_get_state_mixed).
"""
import numpy as np
import torch

from . import _lib
from . import constants as K


def make_config(flags, room_width, room_length, layout='hwc', rotate_rounding='fma'):
    """simaps_config of one configuration.  rotate_rounding: 'fma' / 'plain', how the host the
    reference runs on rounds scipy.ndimage.rotate's out_center (include/simaps.h SIMAPS_ROT_*;
    K.host_rotate_rounding() measures it)."""
    if rotate_rounding not in _lib.ROT_IDS:
        raise ValueError('rotate_rounding must be one of %s' % sorted(_lib.ROT_IDS))
    H, W = K.padded_room_shape(room_width, room_length)
    i0, j0, h, w = K.room_rect(room_width, room_length)
    c = _lib.Config()
    c.H, c.W, c.room_i0, c.room_j0, c.room_h, c.room_w = H, W, i0, j0, h, w
    c.use_robot_map = int(bool(flags['use_robot_map']))
    c.use_distance_to_receptacle_map = int(bool(flags['use_distance_to_receptacle_map']))
    c.use_shortest_path_to_receptacle_map = int(bool(flags['use_shortest_path_to_receptacle_map']))
    c.use_shortest_path_map = int(bool(flags['use_shortest_path_map']))
    c.use_intention_map = int(bool(flags['use_intention_map']))
    c.intention_map_encoding = _lib.ENC_IDS[flags['intention_map_encoding']]
    c.intention_map_line_thickness = int(flags['intention_map_line_thickness'])
    c.use_history_map = int(bool(flags['use_history_map']))
    c.use_intention_channels = int(bool(flags['use_intention_channels']))
    c.intention_channel_spatial = int(flags['intention_channel_encoding'] == 'spatial')
    c.layout_chw = 1 if layout == 'chw' else 0
    c.rotate_rounding = _lib.ROT_IDS[rotate_rounding]
    c.distance_to_receptacle_map_scale = float(flags['distance_to_receptacle_map_scale'])
    c.shortest_path_map_scale = float(flags['shortest_path_map_scale'])
    c.intention_map_scale = float(flags['intention_map_scale'])
    c.intention_channel_nonspatial_scale = float(flags['intention_channel_nonspatial_scale'])
    return c


def pack_descriptors(scenes, agents):
    """Host-side packing of the per-step scene descriptor into the C structs.

    scenes: list of scene dicts (simaps.synthetic format); agents: list of (env_idx, robot_idx).
    Column-wise: one numpy assignment per struct field and one flat float list of all path points
    (a per-robot, per-field loop cost ~4.6 ms for 64 envs x 4 robots, 150x the kernel; this 0.8 ms
    in the dev container)."""
    nr = [len(s['robots']) for s in scenes]
    if nr and max(nr) > _lib.MAX_ROBOTS:
        raise ValueError('at most %d robots per env' % _lib.MAX_ROBOTS)
    rl = [r for s in scenes for r in s['robots']]
    n_rob = len(rl)
    robots = np.zeros(n_rob, dtype=_lib.ROBOT_DTYPE)
    envs = np.zeros(len(scenes), dtype=_lib.ENV_DTYPE)
    envs['num_robots'] = nr
    envs['robot_off'] = np.concatenate([[0], np.cumsum(nr)[:-1]]) if nr else []
    recs = [s['receptacle_position'] for s in scenes]
    envs['has_receptacle'] = [rec is not None for rec in recs]
    envs['receptacle_x'] = [rec[0] if rec is not None else 0.0 for rec in recs]
    envs['receptacle_y'] = [rec[1] if rec is not None else 0.0 for rec in recs]
    # A robot that has not acted yet (Robot.__init__ / reset, envs.py:828-832, 958-963; controller
    # 1373-1376) has target_end_effector_position / waypoint_positions / waypoint_index = None and is
    # idle; the reference never reads them for an idle robot (envs.py:2305, 2363, 2371), so it packs
    # with no target and empty paths (the kernel skips idle robots the same way).
    for r in rl:
        if not r['idle'] and (r['target_ee'] is None or r['waypoint_positions'] is None or r['waypoint_index'] is None):
            raise ValueError('a robot that is not idle needs target_ee, waypoint_positions and waypoint_index')
    if n_rob:
        robots['x'] = [r['position'][0] for r in rl]
        robots['y'] = [r['position'][1] for r in rl]
        robots['heading'] = [r['heading'] for r in rl]
        robots['target_x'] = [r['target_ee'][0] if r['target_ee'] is not None else 0.0 for r in rl]
        robots['target_y'] = [r['target_ee'][1] if r['target_ee'] is not None else 0.0 for r in rl]
        robots['type'] = [_lib.TYPE_IDS[r['type']] for r in rl]
        robots['group_index'] = [r['group_index'] for r in rl]
        robots['lifting'] = [r.get('lift_state') == 'lifting' for r in rl]
        robots['idle'] = [bool(r['idle']) for r in rl]
    # per robot, flattened straight into one list of floats: its intention path
    # [position] + waypoints[idx:-1] + [target_ee] (RobotController.get_intention_path, envs.py:1475-1476),
    # then its reversed history path (waypoints[:idx] + [position])[::-1] (get_history_path, 1478-1479, 2318)
    flat, lens = [], []
    for r in rl:
        pos, wps, idx, tgt = r['position'], r['waypoint_positions'], r['waypoint_index'], r['target_ee']
        if tgt is None or wps is None or idx is None:  # idle, never acted: no paths
            lens += (0, 0)
            continue
        mid = wps[idx:-1]
        flat += (pos[0], pos[1])
        for q in mid:
            flat += (q[0], q[1])
        flat += (tgt[0], tgt[1])
        hist = wps[:idx]
        flat += (pos[0], pos[1])
        for q in reversed(hist):
            flat += (q[0], q[1])
        lens += (len(mid) + 2, len(hist) + 1)
    lens = np.array(lens, dtype=np.int64).reshape(-1, 2)
    if len(lens) and lens.max() > _lib.MAX_PATH:
        raise ValueError('path longer than %d points' % _lib.MAX_PATH)
    offs = np.concatenate([[0], np.cumsum(lens.ravel())[:-1]]).reshape(-1, 2) if len(lens) else lens
    if n_rob:
        robots['intention_off'], robots['intention_len'] = offs[:, 0], lens[:, 0]
        robots['history_off'], robots['history_len'] = offs[:, 1], lens[:, 1]
    paths = np.array(flat if flat else [0.0, 0.0], dtype=np.float64).reshape(-1, 2)
    ag = np.zeros(len(agents), dtype=_lib.AGENT_DTYPE)
    if len(agents):
        ea = np.asarray(agents, dtype=np.int64).reshape(-1, 2)
        ag['env'], ag['robot'], ag['map_slot'] = ea[:, 0], ea[:, 1], np.arange(len(agents))
    return robots, envs, ag, paths


def descriptor_arrays(scenes):
    """The per-step robot state of `scenes` as the arrays StateBatch.set_descriptor_arrays takes
    (what a simulator keeps per robot anyway): pose [R, 3], target [R, 2], idle [R], lifting [R],
    waypoints [R, K, 2] (padded), wp_count [R] (-1: None, never acted), wp_index [R]; R = all
    robots of all scenes in order."""
    rl = [r for s in scenes for r in s['robots']]
    R = len(rl)
    K = max([len(r['waypoint_positions']) for r in rl if r['waypoint_positions'] is not None] + [1])
    out = {'pose': np.zeros((R, 3)), 'target': np.zeros((R, 2)), 'idle': np.zeros(R, bool), 'lifting': np.zeros(R, bool),
           'waypoints': np.zeros((R, K, 2)), 'wp_count': np.full(R, -1, np.int32), 'wp_index': np.zeros(R, np.int32)}
    for k, r in enumerate(rl):
        out['pose'][k] = (r['position'][0], r['position'][1], r['heading'])
        out['idle'][k] = bool(r['idle'])
        out['lifting'][k] = r.get('lift_state') == 'lifting'
        if r['waypoint_positions'] is not None and r['target_ee'] is not None and r['waypoint_index'] is not None:
            out['target'][k] = r['target_ee'][:2]
            w = np.asarray([p[:2] for p in r['waypoint_positions']], dtype=np.float64).reshape(-1, 2)
            out['waypoints'][k, :len(w)] = w
            out['wp_count'][k] = len(w)
            out['wp_index'][k] = r['waypoint_index']
    return out


def resolve_device(device):
    """torch.device with an explicit index ('cuda' -> 'cuda:<current>'), so tensors' devices compare equal."""
    dev = torch.device(device)
    if dev.type == 'cuda' and dev.index is None:
        dev = torch.device('cuda', torch.cuda.current_device())
    return dev


def _to_dev(a, device):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(device)


def launch_stream(device, stream=None):
    """(launch stream, current stream).  A kernel launched on a side stream first waits for the
    current stream (where this module uploads its inputs and allocates its outputs)."""
    cur = torch.cuda.current_stream(device)
    s = cur if stream is None else stream
    if s != cur:
        s.wait_stream(cur)
    return s, cur


def hold(s, cur, *tensors):
    """Keep tensors a launch on side stream `s` reads or writes alive (caching allocator) until `s`
    has finished it.  Consumers on other streams must wait for `s` themselves (torch semantics)."""
    if s != cur:
        for t in tensors:
            if t is not None:
                t.record_stream(s)


class _ArrayUpload:
    """The array fast path of the per-step robot state, shared by StateBatch and
    MixedStateBatch: needs self.device, self.n_robots and self._type_group ([R, 2] int32 robot class
    and group, all robots of all envs in order)."""

    def set_descriptor_arrays(self, pose, target, idle, lifting, waypoints, wp_count, wp_index):
        """Per-step robot state as arrays, all robots of all envs in order (R = robots in the batch;
        shapes as descriptor_arrays() returns, [E, A, ...] accepted): packed into the C structs by
        the native simaps_pack_robots (no per-robot Python), staged in pinned host memory and
        uploaded with ONE asynchronous copy on the current stream.  Robot classes / groups, the envs
        and the agent list are the batch's (fixed at construction); only poses, targets, flags and
        paths change per step."""
        R = self.n_robots
        f64 = lambda a, *shape: np.ascontiguousarray(a, dtype=np.float64).reshape(*shape)  # noqa: E731
        pose, target = f64(pose, R, 3), f64(target, R, 2)
        wps = np.ascontiguousarray(waypoints, dtype=np.float64)
        K = wps.shape[-2] if wps.ndim >= 2 else 0
        wps = wps.reshape(R, K, 2)
        flags = (np.asarray(idle, dtype=np.int32).reshape(R) | (np.asarray(lifting, dtype=np.int32).reshape(R) << 1))
        cnt = np.ascontiguousarray(wp_count, dtype=np.int32).reshape(R)
        idx = np.ascontiguousarray(wp_index, dtype=np.int32).reshape(R)
        if getattr(self, '_stage', None) is None:
            self._rob_bytes = -(-R * _lib.ROBOT_DTYPE.itemsize // 256) * 256
            nb = self._rob_bytes + R * 2 * _lib.MAX_PATH * 16
            # a ring of pinned staging buffers: one is rewritten only after its copy has completed
            self._stage = [torch.empty(max(nb, 256), dtype=torch.uint8).pin_memory() for _ in range(3)]
            self._stage_ev = [None] * 3
            self._stage_k = 0
        k = self._stage_k
        self._stage_k = (k + 1) % len(self._stage)
        if self._stage_ev[k] is not None:
            self._stage_ev[k].synchronize()
        host = self._stage[k]
        hp = host.data_ptr()
        _lib.check(_lib.lib.simaps_pack_robots(
            R, pose.ctypes.data, target.ctypes.data, flags.ctypes.data, self._type_group.ctypes.data,
            wps.ctypes.data if K else None, K, cnt.ctypes.data, idx.ctypes.data, hp, hp + self._rob_bytes))
        dev = torch.empty(host.shape, dtype=torch.uint8, device=self.device)
        dev.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._stage_ev[k] = ev
        self.robots_d = dev[:R * _lib.ROBOT_DTYPE.itemsize]
        self.paths_d = dev[self._rob_bytes:]
        self.pose_host = pose.copy()  # the poses packed above (the caller may update its array in place)


class StateBatch(_ArrayUpload):
    """One configuration's batch of agent-state stacks, resident on `device`.

    layout='chw' (default, device-native: every channel plane is written with full cache lines and is
    what a conv policy consumes) or 'hwc' (the reference's (96, 96, C) memory order).  as_hwc() gives
    the reference's index order as a zero-copy view either way."""

    def __init__(self, scenes, agents=None, device='cuda', layout='chw'):
        if not scenes:
            raise ValueError('a StateBatch needs at least one scene')
        s0 = scenes[0]
        for s in scenes:
            if (s['H'], s['W'], s['room_width'], s['room_length']) != (s0['H'], s0['W'], s0['room_width'], s0['room_length']) \
                    or s['flags'] != s0['flags'] or K.scene_rotate_rounding(s) != K.scene_rotate_rounding(s0):
                raise ValueError('one StateBatch holds one configuration (grid + flags + rotate rounding)')
        if agents is None:
            agents = [(e, a) for e, s in enumerate(scenes) for a in range(len(s['robots']))]
        self.scenes, self.agents, self.device = scenes, list(agents), resolve_device(device)
        if self.device.type != 'cuda':
            raise ValueError('StateBatch renders on a GPU device (got %s); there is no CPU path' % self.device)
        self.flags = s0['flags']
        self.H, self.W = s0['H'], s0['W']
        self.cfg = make_config(self.flags, s0['room_width'], s0['room_length'], layout,
                               K.scene_rotate_rounding(s0))
        self.num_robots = len(s0['robots'])
        if self.flags['use_intention_channels'] and any(len(s['robots']) != self.num_robots for s in scenes):
            raise ValueError('intention channels need the same robot count in every env of a batch')
        self.C = _lib.lib.simaps_num_channels(self.cfg, self.num_robots)
        self.N = len(self.agents)
        occ = np.stack([scenes[e]['occupancy'][a] for e, a in self.agents]).astype(np.uint8)
        ovh = np.stack([scenes[e]['overhead'][a] for e, a in self.agents]).astype(np.float32)
        self.occupancy = torch.from_numpy(occ).to(self.device)
        self.overhead = torch.from_numpy(ovh).to(self.device)
        self.set_descriptors(scenes)
        self.n_robots = sum(len(s['robots']) for s in scenes)
        self._type_group = np.array([(_lib.TYPE_IDS[r['type']], r['group_index']) for s in scenes for r in s['robots']],
                                    dtype=np.int32).reshape(-1, 2)
        self.layout = layout
        # receptacle distance cache (receptacle_distances): one record per map slot, allocated on first
        # use; a record is current while its slot's map version equals the version it was made at
        self._rec = None
        self._map_ver = np.zeros(self.N, dtype=np.int64)
        self._rec_ver = np.full(self.N, -1, dtype=np.int64)
        # slots whose maps a captured ingest graph may change on any replay, unseen by the host
        # versions above: their cached records are never served (always a miss, full SSSP)
        self._replayed = np.zeros(self.N, dtype=bool)
        # the stream of the last launch that wrote or read the cache: a next one on another stream
        # waits for it (_rec_wait)
        self._rec_stream = None

    def set_descriptors(self, scenes):
        """Upload a new per-step scene descriptor (poses, controller state, paths)."""
        robots, envs, ag, paths = pack_descriptors(scenes, self.agents)
        self.scenes = scenes
        if hasattr(self, '_rec_ver'):
            self._rec_ver[:] = -1  # new scenes may move a receptacle: no cached array stays valid
        # per map slot: its env's receptacle (x, y) (receptacle_distances' SSSP source)
        env_of = np.asarray([e for e, _ in self.agents], dtype=np.int64)
        self._slot_has_rec = np.asarray([scenes[e]['receptacle_position'] is not None for e in env_of], dtype=bool)
        self._slot_rec_xy = np.asarray([scenes[e]['receptacle_position'][:2] if scenes[e]['receptacle_position'] is not None
                                        else (0.0, 0.0) for e in env_of], dtype=np.float64).reshape(-1, 2)
        # (ingest takes the camera poses from here)
        self.pose_host = np.stack([robots['x'], robots['y'], robots['heading']], 1) if len(robots) else np.zeros((0, 3))
        self._robot_off = envs['robot_off'].astype(np.int64)
        # one host->device copy for the four arrays (256-B aligned sections of one byte buffer):
        # each small copy costs a driver round trip
        parts = [np.ascontiguousarray(a).view(np.uint8).reshape(-1) for a in (robots, envs, ag, paths)]
        offs = np.concatenate([[0], np.cumsum([-(-p.nbytes // 256) * 256 for p in parts])])
        buf = np.zeros(max(int(offs[-1]), 256), np.uint8)
        for o, p in zip(offs, parts):
            buf[o:o + p.nbytes] = p
        dev = torch.from_numpy(buf).to(self.device)
        self.robots_d, self.envs_d, self.agents_d, self.paths_d = (dev[o:o + p.nbytes] for o, p in zip(offs, parts))
        if not hasattr(self, '_subsets'):
            self._subsets = {}  # subset agent lists depend on self.agents only: kept across steps

    def set_maps(self, occupancy=None, overhead=None, slots=None):
        """Replace the per-agent global maps -- what Mapper.update / OccupancyMap.update produce each
        step (envs.py:2056-2062, 2447-2450) -- for every map slot, or for `slots` only.  Inputs are
        [n, H, W] arrays / tensors (uint8 occupancy, float32 overhead-without-robots)."""
        idx = None if slots is None else torch.as_tensor(list(slots), dtype=torch.long, device=self.device)
        if occupancy is not None:  # the cspace follows the occupancy map: cached receptacle arrays go stale
            self._map_ver[slice(None) if slots is None else np.asarray(list(slots), dtype=np.int64)] += 1
        for name, dst, dt in (('occupancy', self.occupancy, torch.uint8), ('overhead', self.overhead, torch.float32)):
            src = occupancy if name == 'occupancy' else overhead
            if src is None:
                continue
            src = torch.as_tensor(src).to(device=self.device, dtype=dt)
            want = (self.N if idx is None else len(idx), self.H, self.W)
            if tuple(src.shape) != want:
                raise ValueError('%s must have shape %s, got %s' % (name, want, tuple(src.shape)))
            if idx is None:
                dst.copy_(src)
            else:
                dst[idx] = src

    def subset_descriptor(self, slots):
        """Device agent list rendering only map slots `slots` (indices into self.agents), e.g. the
        robots awaiting a new action (envs.py:322-323).  Cached per distinct subset."""
        key = tuple(int(k) for k in slots)
        if len(key) == self.N and key == tuple(range(self.N)):
            return self.agents_d, self.N  # every agent, in order
        d = self._subsets.get(key)
        if d is None:
            ks = np.asarray(key, dtype=np.int64)
            if len(ks) and (ks.min() < 0 or ks.max() >= self.N):
                raise IndexError('map slot %d outside [0, %d)' % (int(ks[(ks < 0) | (ks >= self.N)][0]), self.N))
            ea = np.asarray(self.agents, dtype=np.int64).reshape(-1, 2)[ks] if len(ks) else np.zeros((0, 2), np.int64)
            ag = np.zeros(len(key), dtype=_lib.AGENT_DTYPE)
            ag['env'], ag['robot'], ag['map_slot'] = ea[:, 0], ea[:, 1], ks
            if len(self._subsets) >= 64:  # awaiting patterns vary per step: keep the cache bounded
                self._subsets.clear()
            d = self._subsets[key] = _to_dev(ag, self.device)
        return d, len(key)

    def out_shape(self, n=None):
        n = self.N if n is None else n
        if self.cfg.layout_chw:
            return (n, self.C, K.LOCAL_MAP_PIXEL_WIDTH, K.LOCAL_MAP_PIXEL_WIDTH)
        return (n, K.LOCAL_MAP_PIXEL_WIDTH, K.LOCAL_MAP_PIXEL_WIDTH, self.C)

    def alloc_state(self, n=None):
        return torch.empty(self.out_shape(n), dtype=torch.float32, device=self.device)

    def as_hwc(self, state):
        """The reference's (N, 96, 96, C) view of a rendered batch (zero-copy for the CHW layout)."""
        return state.permute(0, 2, 3, 1) if self.cfg.layout_chw else state

    def alloc_debug(self, n=None):
        n = self.N if n is None else n
        h, w = self.cfg.room_h, self.cfg.room_w
        z = lambda *s, dt: torch.empty(s, dtype=dt, device=self.device)  # noqa: E731
        return {'cspace': z(n, h, w, dt=torch.uint8), 'sources': z(n, 2, 4, dt=torch.int32),
                'dist': z(n, 2, h, w, dt=torch.float32), 'status': z(n, dt=torch.int32)}

    def render(self, out=None, debug=None, stream=None, slots=None):
        """Launch the fused kernel: the stacks of every agent (or of map slots `slots`, in that
        order) into `out` (allocated if None).  Asynchronous on `stream` (default: the current
        stream); with a side stream, wait for it before reading `out` on another stream."""
        agents_d, n = (self.agents_d, self.N) if slots is None else self.subset_descriptor(slots)
        if out is None:
            out = self.alloc_state(n)
        if not (out.is_contiguous() and tuple(out.shape) == self.out_shape(n) and out.dtype == torch.float32
                and out.device == self.device):
            raise ValueError('out must be a contiguous float32 %s tensor on %s' % (self.out_shape(n), self.device))
        if n == 0:
            return out
        dbg = None
        rec = self._rec if self._rec is not None and self.flags['use_shortest_path_to_receptacle_map'] else None
        if debug is not None or rec is not None:
            debug = debug or {}
            for k, v in debug.items():
                if v is not None and (v.shape[0] != n or not v.is_contiguous() or v.device != self.device):
                    raise ValueError('debug[%r] must be contiguous with leading dim %d on %s' % (k, n, self.device))
            dbg = _lib.Debug(*(debug[k].data_ptr() if debug.get(k) is not None else None
                               for k in ('cspace', 'sources', 'dist', 'status')), None if rec is None else rec.data_ptr())
        s, cur = launch_stream(self.device, stream)
        if rec is not None:
            self._rec_wait(s)
        _lib.check(_lib.lib.simaps_get_state(
            self.cfg, n, _lib.ptr(agents_d), _lib.ptr(self.envs_d), _lib.ptr(self.robots_d),
            _lib.ptr(self.paths_d), _lib.ptr(self.occupancy), _lib.ptr(self.overhead), _lib.ptr(out),
            self.num_robots if self.flags['use_intention_channels'] else 0,
            None if dbg is None else dbg, _lib.stream_handle(s)))
        hold(s, cur, out, agents_d, self.envs_d, self.robots_d, self.paths_d, self.occupancy, self.overhead, rec,
             *(debug.values() if debug else ()))
        if rec is not None:
            self._rec_record(s)
        if rec is not None:  # every rendered slot's receptacle array is now its current map's
            sl = np.arange(self.N) if slots is None else np.asarray(list(slots), dtype=np.int64)
            self._rec_ver[sl] = self._map_ver[sl]
        return out


    def shortest_path_distances(self, sources, targets, slots=None, stream=None, _rec=None):
        """OccupancyMap.shortest_path_distance(source, target) (envs.py:2507-2512) on each agent's own
        map: sources [n, 2] and targets [n, Q, 2] fp64 (x, y) positions for map slots `slots` (all
        agents if None) -> [n, Q] float64 device tensor (metres; -1/96 where unreachable)."""
        agents_d, n = (self.agents_d, self.N) if slots is None else self.subset_descriptor(slots)
        src = torch.as_tensor(sources, dtype=torch.float64).to(self.device).contiguous()
        tgt = torch.as_tensor(targets, dtype=torch.float64).to(self.device).contiguous()
        if tuple(src.shape) != (n, 2) or tgt.dim() != 3 or tgt.shape[0] != n or tgt.shape[2] != 2:
            raise ValueError('sources must be [%d, 2] and targets [%d, Q, 2]' % (n, n))
        Q = tgt.shape[1]
        out = torch.empty((n, Q), dtype=torch.float64, device=self.device)
        if n == 0 or Q == 0:
            return out
        s, cur = launch_stream(self.device, stream)
        if _rec is not None:
            self._rec_wait(s)
        _lib.check(_lib.lib.simaps_sp_distance(
            self.cfg, n, _lib.ptr(agents_d), _lib.ptr(self.envs_d), _lib.ptr(self.robots_d), _lib.ptr(self.occupancy),
            _lib.ptr(src), _lib.ptr(tgt), Q, _lib.ptr(out), _lib.ptr(_rec), _lib.stream_handle(s)))
        hold(s, cur, src, tgt, out, agents_d, self.envs_d, self.robots_d, self.occupancy, _rec)
        if _rec is not None:
            self._rec_record(s)
        return out

    def _rec_wait(self, s):
        """Order a launch on stream `s` that writes or reads the receptacle cache after the previous
        such launch (on whatever stream it ran): render() and the miss path write records, the lookup
        reads them, and the caller never sees the buffer to order these itself.  Chained: each user
        waits for the one before, so all of them are ordered.  On the previous user's own stream the
        stream order does it (no event); on another, an event recorded now on that stream (it covers
        the previous user and whatever followed it there).  (Inside a graph capture the capture's own
        stream order applies; an event recorded outside it cannot be waited on.)"""
        prev = self._rec_stream
        if prev is None or prev == s:
            return
        with torch.cuda.stream(s):
            if torch.cuda.is_current_stream_capturing():
                return
        with torch.cuda.stream(prev):
            if torch.cuda.is_current_stream_capturing():
                return
        ev = torch.cuda.Event()
        ev.record(prev)
        s.wait_event(ev)

    def _rec_record(self, s):
        self._rec_stream = s

    def enable_receptacle_cache(self):
        """Allocate the receptacle distance cache (one simaps_rec_cache_bytes record per map slot): from
        now on render() keeps every rendered agent's receptacle array (with
        use_shortest_path_to_receptacle_map) and receptacle_distances() answers from it."""
        if self._rec is None:
            nb = _lib.lib.simaps_rec_cache_bytes(self.cfg)
            _lib.check(min(nb, 0))
            self._rec = torch.empty((self.N, nb), dtype=torch.uint8, device=self.device)
            self._rec_ver[:] = -1
        return self._rec

    def receptacle_distances(self, targets, slots=None, stream=None, cache=True):
        """Mapper.distance_to_receptacle with shortest-path partial rewards (envs.py:2190-2194) on each
        agent's own map: targets [n, Q, 2] fp64 (x, y) for map slots `slots` (all if None) -> [n, Q]
        float64 device tensor (metres; -1/96 unreachable).  Like the reference, which answers from the
        GridGraph cache get_state filled (shortest_paths.pyx:116-119, 156-163): slots whose cached
        receptacle array belongs to their current map (render() since the last map change) are a
        lookup (simaps_sp_lookup); the others run the full SSSP from the receptacle (simaps_sp_distance)
        and keep their array for the next call.  cache=False: always the full SSSP, nothing kept."""
        sl = np.arange(self.N, dtype=np.int64) if slots is None else np.asarray(list(slots), dtype=np.int64)
        n = len(sl)
        tgt = torch.as_tensor(targets, dtype=torch.float64).to(self.device).contiguous()
        if tgt.dim() != 3 or tgt.shape[0] != n or tgt.shape[2] != 2:
            raise ValueError('targets must be [%d, Q, 2]' % n)
        if not self._slot_has_rec[sl].all():
            raise ValueError('distance_to_receptacle needs a receptacle (not a rescue env)')
        if not cache:
            return self.shortest_path_distances(self._slot_rec_xy[sl], tgt, slots=slots, stream=stream)
        rec = self.enable_receptacle_cache()
        hit = (self._rec_ver[sl] == self._map_ver[sl]) & ~self._replayed[sl]
        Q = tgt.shape[1]
        s, cur = launch_stream(self.device, stream)
        with torch.cuda.stream(s):  # (every launch, copy and allocation below on the launch stream)
            out = torch.empty((n, Q), dtype=torch.float64, device=self.device)
            if n == 0 or Q == 0:
                return out
            if hit.all():  # the common case: one lookup launch straight into `out`
                groups = [(None, out)]
            else:
                groups = [(np.nonzero(~hit)[0], None), (np.nonzero(hit)[0], None)]
            for k, (rows, dst) in enumerate(groups):
                if rows is not None and len(rows) == 0:
                    continue
                full = len(groups) == 2 and k == 0  # the misses: full SSSP, arrays into the cache
                sub = None if rows is None else torch.as_tensor(rows, device=self.device)
                th = tgt if sub is None else tgt[sub].contiguous()
                rs_ = sl if rows is None else sl[rows]
                if full:
                    o = self.shortest_path_distances(self._slot_rec_xy[rs_], th, slots=rs_, stream=s, _rec=rec)
                    self._rec_ver[rs_] = self._map_ver[rs_]
                else:
                    agents_d, m = self.subset_descriptor(rs_) if (slots is not None or rows is not None) \
                        else (self.agents_d, self.N)
                    o = dst if dst is not None else torch.empty((m, Q), dtype=torch.float64, device=self.device)
                    self._rec_wait(s)
                    _lib.check(_lib.lib.simaps_sp_lookup(self.cfg, m, _lib.ptr(agents_d), _lib.ptr(rec), _lib.ptr(th),
                                                         Q, _lib.ptr(o), _lib.stream_handle(s)))
                    hold(s, cur, agents_d, th, o)
                    self._rec_record(s)
                if sub is not None:
                    out[sub] = o
        hold(s, cur, rec, tgt, out)
        return out


    # -- OccupancyMap (envs.py:2409-2524) outputs (round 6) ---------------------------------------------
    def scatter_obstacles(self, points, seg, obstacle_seg_value, slots=None, stream=None, out=None):
        """OccupancyMap.update's obstacle scatter (envs.py:2445-2450) into the occupancy maps of map slots
        `slots` (all if None): points [n, P, 3] float32 (x, y, z), seg [n, P] float32 -- every point with
        np.isclose(seg, obstacle_seg_value) marks its pixel occupied.  One launch (simaps_occupancy_scatter).
        out: another [num_map_slots, H, W] uint8 device tensor to mark instead of the occupancy maps (the
        show_map free-space map, OccupancyMap.update 2462-2465)."""
        agents_d, n = (self.agents_d, self.N) if slots is None else self.subset_descriptor(slots)
        pts = torch.as_tensor(points, dtype=torch.float32).to(self.device).reshape(n, -1, 3).contiguous()
        sg = torch.as_tensor(seg, dtype=torch.float32).to(self.device).reshape(n, -1).contiguous()
        if sg.shape[1] != pts.shape[1]:
            raise ValueError('points [n, P, 3] and seg [n, P] must have the same P')
        if out is None:
            out = self.occupancy
        elif (out.dtype != torch.uint8 or tuple(out.shape) != tuple(self.occupancy.shape) or not out.is_contiguous()
              or out.device != self.occupancy.device):
            raise ValueError('out must be a contiguous uint8 %s tensor on %s' % (tuple(self.occupancy.shape), self.device))
        if n == 0 or pts.shape[1] == 0:
            return
        if out is self.occupancy:
            self._map_ver[slice(None) if slots is None else np.asarray(list(slots), dtype=np.int64)] += 1
        s, cur = launch_stream(self.device, stream)
        _lib.check(_lib.lib.simaps_occupancy_scatter(self.cfg, n, _lib.ptr(agents_d), _lib.ptr(pts), _lib.ptr(sg),
                                                     pts.shape[1], float(obstacle_seg_value), _lib.ptr(out),
                                                     _lib.stream_handle(s)))
        hold(s, cur, agents_d, pts, sg, out)

    def build_cspace(self, slots=None, cspace=True, thin=True, stream=None):
        """OccupancyMap.configuration_space / cspace_thin (envs.py:2453, 2456) of map slots `slots` (all
        if None) over the whole grid: (cspace [n, H, W] uint8 or None, cspace_thin [n, H, W] uint8 or
        None) device tensors.  One launch (simaps_build_cspace)."""
        agents_d, n = (self.agents_d, self.N) if slots is None else self.subset_descriptor(slots)
        z = lambda on: torch.empty((n, self.H, self.W), dtype=torch.uint8, device=self.device) if on else None  # noqa: E731
        cs, th = z(cspace), z(thin)
        if n == 0 or (cs is None and th is None):
            return cs, th
        s, cur = launch_stream(self.device, stream)
        _lib.check(_lib.lib.simaps_build_cspace(self.cfg, n, _lib.ptr(agents_d), _lib.ptr(self.envs_d), _lib.ptr(self.robots_d),
                                                _lib.ptr(self.occupancy), _lib.ptr(cs), _lib.ptr(th), _lib.stream_handle(s)))
        hold(s, cur, agents_d, self.occupancy, cs, th)
        return cs, th

    def snap_pixels(self, pixels, slots=None, stream=None):
        """OccupancyMap._closest_valid_cspace_indices (envs.py:2523-2524) = closest_cspace_indices[:, i, j]
        of each agent's own map at query pixels [n, Q, 2] int (i, j) -> [n, Q, 2] int32 device tensor
        ((-1, -1) for pixels outside the grid).  One launch (simaps_snap_sources)."""
        agents_d, n = (self.agents_d, self.N) if slots is None else self.subset_descriptor(slots)
        px = torch.as_tensor(pixels).to(device=self.device, dtype=torch.int32).contiguous()
        if px.dim() != 3 or px.shape[0] != n or px.shape[2] != 2:
            raise ValueError('pixels must be [%d, Q, 2]' % n)
        out = torch.empty(px.shape, dtype=torch.int32, device=self.device)
        Q = px.shape[1]
        if n == 0 or Q == 0:
            return out
        s, cur = launch_stream(self.device, stream)
        _lib.check(_lib.lib.simaps_snap_sources(self.cfg, n, _lib.ptr(agents_d), _lib.ptr(self.envs_d), _lib.ptr(self.robots_d),
                                                _lib.ptr(self.occupancy), _lib.ptr(px), Q, _lib.ptr(out), _lib.stream_handle(s)))
        hold(s, cur, agents_d, self.occupancy, px, out)
        return out

    def global_maps(self, slots=None, stream=None):
        """The whole-grid maps of Mapper.get_state(save_figures=True) (envs.py:2115-2182) for map slots
        `slots` (all if None), one launch (simaps_global_maps): {'overhead': _create_global_overhead_map,
        'robot': _create_global_robot_map(seg=False) (if use_robot_map), 'history' / 'intention':
        _create_global_intention_or_history_map (if use_history_map / use_intention_map)} as [n, H, W]
        float32 device tensors."""
        agents_d, n = (self.agents_d, self.N) if slots is None else self.subset_descriptor(slots)
        z = lambda: torch.empty((n, self.H, self.W), dtype=torch.float32, device=self.device)  # noqa: E731
        out = {'overhead': z()}
        if self.flags['use_robot_map']:
            out['robot'] = z()
        if self.flags['use_history_map']:
            out['history'] = z()
        if self.flags['use_intention_map']:
            out['intention'] = z()
        if n == 0:
            return out
        s, cur = launch_stream(self.device, stream)
        _lib.check(_lib.lib.simaps_global_maps(self.cfg, n, _lib.ptr(agents_d), _lib.ptr(self.envs_d), _lib.ptr(self.robots_d),
                                               _lib.ptr(self.paths_d), _lib.ptr(self.overhead), _lib.ptr(out['overhead']),
                                               _lib.ptr(out.get('robot')), _lib.ptr(out.get('history')),
                                               _lib.ptr(out.get('intention')), _lib.stream_handle(s)))
        hold(s, cur, agents_d, self.envs_d, self.robots_d, self.paths_d, self.overhead, *out.values())
        return out

    def shortest_path_images(self, positions, slots=None):
        """OccupancyMap.shortest_path_image(position) (envs.py:2514-2517) of each agent's own map:
        positions [n, 2] (x, y) -> [n, H, W] float32 device tensor of distances / 96 (-1 / 96 where
        unreachable): simaps_build_cspace + simaps_snap_sources + simaps_sssp_grid, three launches."""
        sl = list(range(self.N)) if slots is None else [int(k) for k in slots]
        n = len(sl)
        cs, _ = self.build_cspace(slots=slots, thin=False)
        px = np.array([K.position_to_pixel_indices(float(x), float(y), (self.H, self.W)) for x, y in np.asarray(positions)[:, :2]],
                      dtype=np.int32).reshape(n, 1, 2)
        src = self.snap_pixels(px, slots=slots)[:, 0, :]
        i0, j0, h, w = self.cfg.room_i0, self.cfg.room_j0, self.cfg.room_h, self.cfg.room_w
        img = sssp_grid(cs, src, window=(i0, j0, h, w))
        return img / np.float32(K.LOCAL_MAP_PIXELS_PER_METER)

    def shortest_paths(self, sources, targets, slots=None, max_points=64, stream=None):
        """OccupancyMap.shortest_path(source, target) (envs.py:2478-2505) on each agent's own map:
        sources / targets [n, 2] fp64 (x, y) for map slots `slots` (all agents if None) -> list of n
        waypoint lists [(x, y, 0), ...] like the reference returns (Robot.store_new_action,
        envs.py:875-876)."""
        n = self.N if slots is None else len(slots)
        if n == 0:
            return []
        s, cur = launch_stream(self.device, stream)
        xy, cnt = self.launch_shortest_paths(sources, targets, slots, max_points, stream)
        if s != cur:
            cur.wait_stream(s)
        xy, cnt = xy.cpu().numpy(), cnt.cpu().numpy()
        _lib.check_faults()
        if (cnt < 0).any():
            raise RuntimeError('a path has %d waypoints > max_points=%d' % (-cnt.min(), max_points))
        return _point_lists(xy, cnt, 0)


    def launch_shortest_paths(self, sources, targets, slots=None, max_points=64, stream=None):
        """The device half of shortest_paths(): one launch, results left on the device as
        (xy [n, max_points, 2] fp64, count [n] int32; count = -needed if max_points is too small)."""
        agents_d, n = (self.agents_d, self.N) if slots is None else self.subset_descriptor(slots)
        src = torch.as_tensor(sources, dtype=torch.float64).to(self.device).contiguous()
        tgt = torch.as_tensor(targets, dtype=torch.float64).to(self.device).contiguous()
        if tuple(src.shape) != (n, 2) or tuple(tgt.shape) != (n, 2):
            raise ValueError('sources and targets must be [%d, 2]' % n)
        xy = torch.empty((n, max_points, 2), dtype=torch.float64, device=self.device)
        cnt = torch.empty((n,), dtype=torch.int32, device=self.device)
        if n == 0:
            return xy, cnt
        s, cur = launch_stream(self.device, stream)
        _lib.check(_lib.lib.simaps_shortest_path(
            self.cfg, n, _lib.ptr(agents_d), _lib.ptr(self.envs_d), _lib.ptr(self.robots_d), _lib.ptr(self.occupancy),
            _lib.ptr(src), _lib.ptr(tgt), max_points, _lib.ptr(xy), _lib.ptr(cnt), _lib.stream_handle(s)))
        hold(s, cur, src, tgt, xy, cnt, agents_d, self.envs_d, self.robots_d, self.occupancy)
        return xy, cnt

    def ingest(self, depth, seg_raw, camera='forward', slots=None, seg_ids=None, stream=None):
        """Robot.update_map minus the simulator (envs.py:925, 2056-2066) for map slots `slots` (all
        agents if None): each robot's camera frame -- depth buffer [n, Hc, Wc] float32 and
        segmentation body ids [n, Hc, Wc] int32, as pybullet getCameraImage returns them -- becomes a
        point cloud that updates the robot's overhead and occupancy maps in place on the device.
        camera: 'forward' (use_partial_observations) or 'overhead'; seg_ids: per-env dict of body ids
        (default: the synthetic scenes' ids).  The camera pose comes from the current descriptor."""
        self.launch_ingest(self.prepare_ingest(depth, seg_raw, camera, slots, seg_ids), stream)

    def prepare_ingest(self, depth, seg_raw, camera='forward', slots=None, seg_ids=None):
        """The host half of ingest(): uploads the frames and packs the camera poses / body ids once;
        launch_ingest() replays the device half (what tools/bench_extra.py times alone)."""
        from . import camera as cam_mod, synthetic
        spec = cam_mod.CAMERAS[camera]
        agents_d, n = (self.agents_d, self.N) if slots is None else self.subset_descriptor(slots)
        idx = list(range(self.N)) if slots is None else [int(k) for k in slots]
        if len(set(idx)) != len(idx):
            raise ValueError('one frame per map slot and launch (slots repeat)')
        dep = torch.as_tensor(depth).to(device=self.device, dtype=torch.float32).contiguous()
        seg = torch.as_tensor(seg_raw).to(device=self.device, dtype=torch.int32).contiguous()
        want = (n, spec.height_px, spec.width_px)
        if tuple(dep.shape) != want or tuple(seg.shape) != want:
            raise ValueError('depth and seg_raw must be %s' % (want,))
        poses = [self.pose_host[self._robot_off[e] + a] for e, a in (self.agents[k] for k in idx)]
        params = spec.params_batch(poses).reshape(n, 9)
        ids = np.zeros(len(self.scenes), dtype=_lib.SEG_IDS_DTYPE)
        for f in ('min_obstacle', 'max_obstacle', 'receptacle', 'min_cube', 'max_cube'):
            ids[f] = [seg_ids[e][f] for e in range(len(self.scenes))] if seg_ids is not None else synthetic.SEG_IDS[f]
        ids['has_receptacle'] = [sc['receptacle_position'] is not None for sc in self.scenes]
        if getattr(self, '_keys', None) is None:  # (epoch-tagged from here on: launch_ingest)
            self._keys = torch.zeros((self.N, self.H, self.W), dtype=torch.int64, device=self.device)
            self._epoch = 0
        nch = _lib.lib.simaps_ingest_chunks(spec.height_px, spec.width_px)  # point-pass chunks per frame
        if nch < 0:
            _lib.check(nch)
        nbox = n * nch * 4
        if getattr(self, '_boxes', None) is None or self._boxes.numel() < nbox:
            self._boxes = torch.empty((nbox,), dtype=torch.int32, device=self.device)
        cam = _lib.Camera(spec.height_px, spec.width_px, spec.near, spec.far, spec.cx2, spec.cy2)
        return {'n': n, 'slots': np.asarray(idx, dtype=np.int64), 'cam': cam, 'agents': agents_d,
                'ids': _to_dev(ids, self.device),
                'params': torch.from_numpy(params).to(self.device), 'depth': dep, 'seg': seg}

    def reset_ingest_keys(self, stream=None):
        """Zero the ingest key map now (on `stream`).  Call it before capturing ingest() into a CUDA
        graph after eager ingests: otherwise the capture has to include that zeroing, and every
        replay pays it."""
        if getattr(self, '_keys', None) is None:
            return
        s, cur = launch_stream(self.device, stream)
        self._wait_last_ingest(s)
        with torch.cuda.stream(s):
            self._keys.zero_()
        hold(s, cur, self._keys)
        self._epoch = 0

    def _wait_last_ingest(self, s):
        """Before the key map is zeroed on stream `s`: the last eager ingest launch may still use it
        on another stream -- wait for an event recorded now on that stream (on the same stream,
        stream order suffices)."""
        prev = getattr(self, '_ingest_stream', None)
        if prev is None or prev == s:
            return
        ev = torch.cuda.Event()
        ev.record(prev)
        s.wait_event(ev)

    def launch_ingest(self, prep, stream=None):
        if prep['n'] == 0:
            return
        self._map_ver[prep['slots']] += 1  # (the receptacle cache of these slots goes stale)
        s, cur = launch_stream(self.device, stream)
        with torch.cuda.stream(s):
            capturing = torch.cuda.is_current_stream_capturing()
        # The key map's launch epoch (include/simaps.h simaps_ingest).  Eager launches count 1..255;
        # at the wrap the map is zeroed on the launch stream first (after the last launch that used
        # it) and the count restarts.  A launch captured into a graph replays its epoch, so it takes
        # the zeroing mode (epoch 0: the map is all zero before and after the launch); once one was
        # captured, the eager launches take it too, since a replay may follow any of them.
        if capturing:
            self._zero_mode = True
            self._replayed[prep['slots']] = True  # (replays change these maps with no host version bump)
        if getattr(self, '_zero_mode', False):
            if getattr(self, '_epoch', 0) != 0:  # keys of earlier eager launches (captured: every replay)
                self._wait_last_ingest(s)
                with torch.cuda.stream(s):
                    self._keys.zero_()
            self._epoch = epoch = 0
        else:
            self._epoch = getattr(self, '_epoch', 0) + 1
            if self._epoch > 255:
                self._wait_last_ingest(s)
                with torch.cuda.stream(s):
                    self._keys.zero_()
                self._epoch = 1
            epoch = self._epoch
        _lib.check(_lib.lib.simaps_ingest(
            self.cfg, prep['cam'], prep['n'], _lib.ptr(prep['agents']), _lib.ptr(prep['ids']), _lib.ptr(prep['params']),
            _lib.ptr(prep['depth']), _lib.ptr(prep['seg']), _lib.ptr(self.overhead), _lib.ptr(self.occupancy),
            _lib.ptr(self._keys), _lib.ptr(self._boxes), epoch, _lib.stream_handle(s)))
        if not capturing:
            self._ingest_stream = s
        hold(s, cur, prep['ids'], prep['params'], prep['depth'], prep['seg'], prep['agents'], self.overhead,
             self.occupancy, self._keys, self._boxes)


def _point_lists(pts, cnt, *extra):
    """pts [n, m, 2] (NumPy), cnt [n] >= 0 -> n lists of tuples (p0, p1, *extra) of Python scalars.
    One tolist() of the valid points instead of a NumPy scalar conversion per point (256 paths:
    2.4 -> 0.3 ms in the dev container)."""
    m = int(cnt.max()) if len(cnt) else 0
    valid = np.arange(m)[None, :] < cnt[:, None]
    p0, p1 = pts[:, :m, 0][valid].tolist(), pts[:, :m, 1][valid].tolist()
    flat = list(zip(p0, p1, *[[e] * len(p0) for e in extra]))
    out, o = [], 0
    for k in cnt.tolist():
        out.append(flat[o:o + k])
        o += k
    return out


def sssp_grid(grids, sources, window=None, stream=None):
    """Batched GridGraph(grid).shortest_path_image(source) on device.

    grids: uint8 tensor [B, H, W] (device), sources: int32 [B, 2].  window = (i0, j0, h, w) that
    contains every free cell (defaults to the whole grid).  Windows beyond the LDS-resident limit
    run the global-memory kernels (same results)."""
    B, H, W = grids.shape
    if window is None:
        window = (0, 0, H, W)
    out = torch.empty((B, H, W), dtype=torch.float32, device=grids.device)
    src = sources.to(device=grids.device, dtype=torch.int32).contiguous()
    g = grids.contiguous()
    s, cur = launch_stream(grids.device, stream)
    _lib.check(_lib.lib.simaps_sssp_grid(B, H, W, _lib.ptr(g), _lib.ptr(src), _lib.ptr(out),
                                         *[int(x) for x in window], _lib.stream_handle(s)))
    hold(s, cur, g, src, out)
    return out


def launch_grid_paths(grids, sources, targets, window=None, max_points=256, stream=None):
    """The device half of grid_paths(): one call, results left on the device as (ij [B, max_points, 2]
    int32, count [B] int32; count = -needed if max_points is too small)."""
    B, H, W = grids.shape
    if window is None:
        window = (0, 0, H, W)
    src = torch.as_tensor(sources).to(device=grids.device, dtype=torch.int32).contiguous()
    tgt = torch.as_tensor(targets).to(device=grids.device, dtype=torch.int32).contiguous()
    if tuple(src.shape) != (B, 2) or tuple(tgt.shape) != (B, 2):
        raise ValueError('sources and targets must be [%d, 2]' % B)
    ij = torch.empty((B, max_points, 2), dtype=torch.int32, device=grids.device)
    cnt = torch.empty((B,), dtype=torch.int32, device=grids.device)
    if B == 0:
        return ij, cnt
    g = grids.contiguous()
    s, cur = launch_stream(grids.device, stream)
    _lib.check(_lib.lib.simaps_grid_path(B, H, W, _lib.ptr(g), _lib.ptr(src), _lib.ptr(tgt), *[int(x) for x in window],
                                         max_points, _lib.ptr(ij), _lib.ptr(cnt), _lib.stream_handle(s)))
    hold(s, cur, g, src, tgt, ij, cnt)
    return ij, cnt


def grid_paths(grids, sources, targets, window=None, max_points=256, stream=None, grow=False):
    """Batched GridGraph(grid).shortest_path(source, target) (pyx:121-154) on device.

    grids: uint8 tensor [B, H, W] (device), sources / targets: int [B, 2] cells.  Returns B lists of
    (row, col) waypoints, source first, exactly the reference's (same SPFA parents).  A path with
    more than max_points waypoints raises RuntimeError, or with grow=True is run again with room for
    the longest one (the reference's lists have no limit)."""
    B = grids.shape[0]
    if B == 0:
        return []
    ij, cnt = launch_grid_paths(grids, sources, targets, window, max_points, stream)
    s, cur = launch_stream(grids.device, stream)
    if s != cur:
        cur.wait_stream(s)
    ij, cnt = ij.cpu().numpy(), cnt.cpu().numpy()
    _lib.check_faults()
    if (cnt < 0).any():
        if grow:
            return grid_paths(grids, sources, targets, window, int(-cnt.min()), stream, grow=False)
        raise RuntimeError('a path has %d waypoints > max_points=%d' % (-cnt.min(), max_points))
    return _point_lists(ij, cnt)


def config_key(scene):
    """What one launch of simaps_get_state shares: grid, room, flags and the rotate rounding."""
    return (scene['H'], scene['W'], scene['room_width'], scene['room_length'],
            tuple(sorted(scene['flags'].items())), K.scene_rotate_rounding(scene))


def mixed_key(scene):
    """One entry of a mixed launch's configuration table: config_key, plus the robot count when
    intention channels are on (their number follows it, simaps_num_channels)."""
    return config_key(scene) + ((len(scene['robots']) if scene['flags']['use_intention_channels'] else None),)


def plan_mixed(scenes, layout='chw'):
    """Host plan of a mixed-configuration launch (simaps_get_state_mixed): the distinct table
    entries (mixed_key) in order of first appearance (at most _lib.MAX_MIXED), each env's entry, and
    for agent n = (env e, robot a) in scene order: its entry, its map slot's element offset (slot n;
    maps of H x W of its configuration, back to back) and its stack's float offset (96 * 96 * C of
    its entry, back to back)."""
    keys, cfg_of_env = [], []
    for s in scenes:
        k = mixed_key(s)
        if k not in keys:
            keys.append(k)
        cfg_of_env.append(keys.index(k))
    if len(keys) > _lib.MAX_MIXED:
        raise ValueError('at most %d configurations per mixed launch (got %d)' % (_lib.MAX_MIXED, len(keys)))
    first = [cfg_of_env.index(k) for k in range(len(keys))]
    cfgs, nrs, chans = [], [], []
    for k, e0 in enumerate(first):
        s0 = scenes[e0]
        nr = len(s0['robots'])
        c = make_config(s0['flags'], s0['room_width'], s0['room_length'], layout, K.scene_rotate_rounding(s0))
        cfgs.append(c)
        nrs.append(nr if s0['flags']['use_intention_channels'] else 0)
        chans.append(_lib.lib.simaps_num_channels(c, nr))
    agents = [(e, a) for e, s in enumerate(scenes) for a in range(len(s['robots']))]
    agent_cfg = np.array([cfg_of_env[e] for e, _ in agents], dtype=np.int32)
    hw = np.array([scenes[e]['H'] * scenes[e]['W'] for e, _ in agents], dtype=np.int64)
    per = np.array([K.LOCAL_MAP_PIXEL_WIDTH ** 2 * chans[k] for k in agent_cfg], dtype=np.int64)
    map_off = np.concatenate([[0], np.cumsum(hw)[:-1]]).astype(np.int64) if len(hw) else hw
    out_off = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.int64) if len(per) else per
    return {'cfgs': cfgs, 'num_robots': nrs, 'channels': chans, 'cfg_of_env': cfg_of_env, 'agents': agents,
            'agent_cfg': agent_cfg, 'map_off': map_off, 'map_numel': int(hw.sum()), 'out_off': out_off,
            'out_numel': int(per.sum())}


class MixedStateBatch(_ArrayUpload):
    """Envs of several configurations (grid, room, flags, rotate rounding, and with intention
    channels the robot count; at most _lib.MAX_MIXED) rendered in ONE launch (simaps_get_state_mixed)
    -- e.g. the envs of collectors of different configurations (the reference's collector runs all
    its workers on one, train_multiprocess.py:159-166, 217-228).  Every agent of every scene
    is a map slot, in scene order.  render() returns one flat float32 tensor; states() gives each
    agent's (C, 96, 96) (layout 'chw') or (96, 96, C) ('hwc') view of it, C that of its own
    configuration.  The results equal one StateBatch.render per configuration, bit for bit."""

    def __init__(self, scenes, device='cuda', layout='chw'):
        if not scenes:
            raise ValueError('a MixedStateBatch needs at least one scene')
        if layout not in ('chw', 'hwc'):
            raise ValueError('layout must be chw or hwc')
        self.device = resolve_device(device)
        if self.device.type != 'cuda':
            raise ValueError('MixedStateBatch renders on a GPU device (got %s); there is no CPU path' % self.device)
        self.layout = layout
        self.plan = plan_mixed(scenes, layout)
        self.scenes, self.agents, self.N = scenes, self.plan['agents'], len(self.plan['agents'])
        occ = np.concatenate([np.asarray(scenes[e]['occupancy'][a], dtype=np.uint8).ravel() for e, a in self.agents])
        ovh = np.concatenate([np.asarray(scenes[e]['overhead'][a], dtype=np.float32).ravel() for e, a in self.agents])
        self.occupancy = torch.from_numpy(occ).to(self.device)
        self.overhead = torch.from_numpy(ovh).to(self.device)
        self._cfgs = (_lib.Config * len(self.plan['cfgs']))(*self.plan['cfgs'])
        self._nrs = np.asarray(self.plan['num_robots'], dtype=np.int32)
        self.n_robots = sum(len(s['robots']) for s in scenes)
        self._type_group = np.array([(_lib.TYPE_IDS[r['type']], r['group_index']) for s in scenes for r in s['robots']],
                                    dtype=np.int32).reshape(-1, 2)
        self.agent_cfg_d = torch.from_numpy(self.plan['agent_cfg']).to(self.device)
        self.map_off_d = torch.from_numpy(self.plan['map_off']).to(self.device)
        self.out_off_d = torch.from_numpy(self.plan['out_off']).to(self.device)
        self.set_descriptors(scenes)

    def set_descriptors(self, scenes):
        """Upload a new per-step scene descriptor (poses, controller state, paths) of the same envs."""
        if [mixed_key(s) for s in scenes] != [mixed_key(s) for s in self.scenes]:
            raise ValueError('set_descriptors: the envs and their configurations are fixed at construction')
        robots, envs, ag, paths = pack_descriptors(scenes, self.agents)
        self.scenes = scenes
        self.robots_d, self.envs_d, self.agents_d, self.paths_d = (_to_dev(x, self.device) for x in (robots, envs, ag, paths))

    def alloc_state(self):
        return torch.empty((self.plan['out_numel'],), dtype=torch.float32, device=self.device)

    def render(self, out=None, stream=None):
        """One launch for every agent; asynchronous on `stream` (default: the current stream)."""
        if out is None:
            out = self.alloc_state()
        if not (out.is_contiguous() and out.dtype == torch.float32 and out.numel() == self.plan['out_numel']
                and out.device == self.device):
            raise ValueError('out must be a contiguous float32 tensor of %d elements on %s' % (self.plan['out_numel'], self.device))
        s, cur = launch_stream(self.device, stream)
        _lib.check(_lib.lib.simaps_get_state_mixed(
            self._cfgs, self._nrs.ctypes.data, len(self.plan['cfgs']), self.N, _lib.ptr(self.agents_d),
            _lib.ptr(self.agent_cfg_d), _lib.ptr(self.envs_d), _lib.ptr(self.robots_d), _lib.ptr(self.paths_d),
            _lib.ptr(self.occupancy), _lib.ptr(self.map_off_d), _lib.ptr(self.overhead), _lib.ptr(out),
            _lib.ptr(self.out_off_d), _lib.stream_handle(s)))
        hold(s, cur, out, self.agents_d, self.agent_cfg_d, self.envs_d, self.robots_d, self.paths_d, self.occupancy,
             self.map_off_d, self.overhead, self.out_off_d)
        return out

    def set_maps(self, occupancy=None, overhead=None, slots=None):
        """Replace the global maps (Mapper.update / OccupancyMap.update, envs.py:2056-2062, 2447-2450)
        of every map slot, or of `slots` only: one [H, W] map per slot, of its own configuration's
        grid (uint8 occupancy, float32 overhead-without-robots), arrays or tensors.  One upload per
        argument; the copies are ordered on the current stream like StateBatch.set_maps."""
        slots = list(range(self.N)) if slots is None else [int(k) for k in slots]
        if any(k < 0 or k >= self.N for k in slots):
            raise ValueError('slots must lie in [0, %d)' % self.N)
        shapes = [(self.scenes[self.agents[k][0]]['H'], self.scenes[self.agents[k][0]]['W']) for k in slots]
        for name, src, dst, dt in (('occupancy', occupancy, self.occupancy, torch.uint8),
                                   ('overhead', overhead, self.overhead, torch.float32)):
            if src is None:
                continue
            if len(src) != len(slots):
                raise ValueError('%s: one map per slot (%d), got %d' % (name, len(slots), len(src)))
            parts = [torch.as_tensor(m) for m in src]
            for k, m, hw in zip(slots, parts, shapes):
                if tuple(m.shape) != hw:
                    raise ValueError('%s of slot %d must have shape %s, got %s' % (name, k, hw, tuple(m.shape)))
            flat = torch.cat([m.reshape(-1).to(dt) for m in parts]).to(self.device)
            if slots == list(range(self.N)):
                dst.copy_(flat)
            else:
                off = self.plan['map_off']
                idx = torch.from_numpy(np.concatenate([np.arange(off[k], off[k] + h * w) for k, (h, w) in
                                                       zip(slots, shapes)])).to(self.device)
                dst[idx] = flat

    def states(self, out):
        """Per-agent views of a rendered flat tensor, in agent order."""
        L = K.LOCAL_MAP_PIXEL_WIDTH
        views = []
        for n in range(self.N):
            C = self.plan['channels'][self.plan['agent_cfg'][n]]
            o = int(self.plan['out_off'][n])
            v = out[o:o + L * L * C]
            views.append(v.view(C, L, L) if self.layout == 'chw' else v.view(L, L, C))
        return views
