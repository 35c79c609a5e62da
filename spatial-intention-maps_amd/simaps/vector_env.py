"""Drop-in host interface for the observation path: VectorEnv.get_state() and GridGraph.

The reference calls the path through Python methods:

  VectorEnv.get_state(all_robots=False, save_figures=False)          envs.py:322-323
      -> [[robot.get_state() if robot.awaiting_new_action or all_robots else None
           for robot in robot_group] for robot_group in self.robot_groups]
  Robot.get_state() -> Mapper.get_state() -> (96, 96, C) float32 HWC   envs.py:928-929, 2068-2185
  GridGraph(grid).shortest_path_image(src) / shortest_path_distance    shortest_paths.pyx:24-67, 156-167

VectorEnvObservations keeps that return structure for a batch of E envs of one configuration
(one list-of-lists per env) and renders every requested stack in ONE launch of the fused HIP
kernel (simaps_get_state).  The per-agent maps (OccupancyMap.occupancy_map and
Mapper.global_overhead_map_without_robots) stay resident on the device across steps; per step
only the scene descriptor (poses, controller state, paths) is uploaded.  There is no CPU
fallback: constructing either class without libsimaps.so / a GPU raises.
"""
import numpy as np
import torch

from . import _lib
from . import batch as _batch


def robot_groups(scene):
    """VectorEnv.robot_groups (envs.py:486-496): robot indices grouped by group_index, in order."""
    ng = 1 + max(r['group_index'] for r in scene['robots'])
    groups = [[] for _ in range(ng)]
    for k, r in enumerate(scene['robots']):
        groups[r['group_index']].append(k)
    return groups


class VectorEnvObservations:
    """The observation half of E VectorEnvs of one configuration, device-resident.

    scenes: list of scene dicts (simaps.synthetic format: flags, grid, robots with poses /
    controller state / paths, receptacle, per-agent occupancy + overhead maps).
    layout: 'hwc' returns (96, 96, C) stacks exactly like the reference; 'chw' renders
    (C, 96, 96) planes (what a conv policy consumes, policies.py:44-45) -- states returned by
    get_state() are always the reference's (96, 96, C) index order (views for 'chw')."""

    def __init__(self, scenes, device='cuda', layout='hwc', reuse_outputs=0):
        """reuse_outputs=R > 0: all-robots get_state() renders into a ring of R preallocated output
        batches and returns a structure of views built once per ring slot (no per-call allocation
        or per-robot view creation: ~0.2 ms of host time per 256 stacks).  The states of a call are
        then overwritten R calls later -- copy what must live longer (the reference returns fresh
        arrays; the default R = 0 keeps that).  With numpy=True the ring slots also hold a pinned
        host copy: one asynchronous device->host copy per call into page-locked memory, returned as
        NumPy views (a fresh pageable copy per call otherwise)."""
        self.batch = _batch.StateBatch(scenes, device=device, layout=layout)
        self._ring = [None] * int(reuse_outputs)
        self._ring_k = 0
        self._hring = [None] * int(reuse_outputs)  # (device batch, pinned host batch, NumPy views)
        self._hring_k = 0
        self.groups = [robot_groups(s) for s in scenes]
        self.slot = {ea: n for n, ea in enumerate(self.batch.agents)}
        self.num_envs = len(scenes)
        # [env][group] -> map slots of the group's robots (the all-robots get_state structure)
        self._all_slots = [[[self.slot[(e, a)] for a in g] for g in self.groups[e]] for e in range(self.num_envs)]

    # -- per-step inputs -------------------------------------------------------------------------
    def update(self, scenes=None, occupancy=None, overhead=None, slots=None):
        """New scene descriptors (robot poses, lift state, idle flags, paths, receptacle) and/or
        new per-agent maps for every slot or for map slots `slots` (Robot.update_map, envs.py:925)."""
        if scenes is not None:
            if len(scenes) != self.num_envs or any(len(s['robots']) != len(o['robots'])
                                                   for s, o in zip(scenes, self.batch.scenes)):
                raise ValueError('update() keeps the batch shape: same envs, same robots per env')
            self.batch.set_descriptors(scenes)
        if occupancy is not None or overhead is not None:
            self.batch.set_maps(occupancy, overhead, slots)

    def update_arrays(self, pose, target, idle, lifting, waypoints, wp_count, wp_index):
        """update() from per-robot arrays instead of scene dicts (the fast path: native packing,
        one pinned asynchronous upload); see StateBatch.set_descriptor_arrays / batch.descriptor_arrays."""
        self.batch.set_descriptor_arrays(pose, target, idle, lifting, waypoints, wp_count, wp_index)

    def update_map(self, robots, depth, seg_raw, camera='forward', seg_ids=None, stream=None):
        """Robot.update_map() (envs.py:925-926) for the robots `robots` ([(env, robot), ...], distinct)
        from their camera frames (depth buffer [n, Hc, Wc] float32, segmentation body ids [n, Hc, Wc]):
        one simaps_ingest launch updates their overhead / occupancy maps in place on the device, with
        the camera poses of the current descriptor.  Called for every robot by VectorEnv.reset()
        (envs.py:214-215), for the awaiting robots at the end of VectorEnv.step() (277-280), and for
        a single moving robot every 200 simulation steps by RobotController.step (1401-1403) --
        successive calls apply in order (stream order)."""
        self.batch.ingest(depth, seg_raw, camera=camera, slots=[self.slot[(e, a)] for e, a in robots],
                          seg_ids=seg_ids, stream=stream)

    # -- VectorEnv.get_state ---------------------------------------------------------------------
    def get_state(self, all_robots=False, awaiting=None, save_figures=False, numpy=False, stream=None,
                  figures_dir='figures', occupancy_maps=None):
        """[env][group][robot] -> (96, 96, C) float32 state, or None for robots not awaiting a new
        action (envs.py:322-323).  awaiting: per env, per robot truthy flags
        (robot.awaiting_new_action); None means every robot.  numpy=True returns host NumPy arrays
        like the reference (one device->host copy for the whole batch); otherwise device tensors.
        save_figures=True also writes, for every robot returned, Mapper.get_state's map PNGs
        (envs.py:2115-2182) into figures_dir/robot_id_<id>/ (<id>: the scene robot's 'id' if it has
        one -- the reference's pybullet body id --, else <env>_<robot>), from device-exported global
        maps (simaps.figures; env.png, the simulator's camera image, is not written).  occupancy_maps:
        {(env, robot): OccupancyMap(show_map=True)}, the env.show_occupancy_maps case (envs.py:2180-2182):
        each figured robot's map figure is saved there as global-occupancy-map.png."""
        if save_figures:
            return self._get_state_with_figures(all_robots, awaiting, numpy, stream, figures_dir, occupancy_maps)
        if (all_robots or awaiting is None) and self._ring and not numpy:
            k = self._ring_k
            self._ring_k = (k + 1) % len(self._ring)
            if self._ring[k] is None:
                buf = self.batch.alloc_state()
                rows = self.batch.as_hwc(buf).unbind(0)
                self._ring[k] = (buf, [[[rows[q] for q in g] for g in env] for env in self._all_slots])
            buf, views = self._ring[k]
            self.batch.render(out=buf, stream=stream)
            return views
        if (all_robots or awaiting is None) and self._hring and numpy:
            k = self._hring_k
            self._hring_k = (k + 1) % len(self._hring)
            if self._hring[k] is None:
                buf = self.batch.alloc_state()
                host = torch.empty(buf.shape, dtype=buf.dtype, pin_memory=True)
                rows = self.batch.as_hwc(host).numpy()
                self._hring[k] = (buf, host, [[[rows[q] for q in g] for g in env] for env in self._all_slots])
            buf, host, views = self._hring[k]
            s = stream if stream is not None else torch.cuda.current_stream(self.batch.device)
            self.batch.render(out=buf, stream=s)
            with torch.cuda.stream(s):
                host.copy_(buf, non_blocking=True)
            s.synchronize()
            _lib.check_faults()  # the copy completed: a faulting launch raises here
            return views
        if all_robots or awaiting is None:  # every robot: the batch's own agent list, structure precomputed
            out = self.batch.as_hwc(self.batch.render(stream=stream))
            if numpy:
                if stream is not None:
                    torch.cuda.current_stream(self.batch.device).wait_stream(stream)
                out = out.cpu().numpy()
                _lib.check_faults()
            rows = out if numpy else out.unbind(0)
            return [[[rows[k] for k in g] for g in env] for env in self._all_slots]
        want = []
        for e, s in enumerate(self.batch.scenes):
            for a in range(len(s['robots'])):
                if awaiting[e][a]:
                    want.append(self.slot[(e, a)])
        out = self.batch.as_hwc(self.batch.render(slots=want, stream=stream))
        if numpy:
            if stream is not None:
                torch.cuda.current_stream(self.batch.device).wait_stream(stream)
            out = out.cpu().numpy()
            _lib.check_faults()  # the copy synchronised: a faulting launch raises here
        pos = {k: n for n, k in enumerate(want)}
        rows = out if numpy else out.unbind(0)  # one C++ call for all views (per-item indexing: ~10 us each)
        res = []
        for e in range(self.num_envs):
            res.append([[rows[pos[self.slot[(e, a)]]] if self.slot[(e, a)] in pos else None for a in g]
                        for g in self.groups[e]])
        return res


    def _get_state_with_figures(self, all_robots, awaiting, numpy, stream, figures_dir, occupancy_maps):
        import os
        from . import figures
        states = self.get_state(all_robots, awaiting, numpy=numpy, stream=stream)
        if stream is not None:
            torch.cuda.current_stream(self.batch.device).wait_stream(stream)
        todo = [(e, a, st) for e, env in enumerate(states) for grp, g in zip(env, self.groups[e])
                for a, st in zip(g, grp) if st is not None]
        if not todo:
            return states
        slots = [self.slot[(e, a)] for e, a, _ in todo]
        pos = [self.batch.scenes[e]['robots'][a]['position'][:2] for e, a, _ in todo]
        maps = figures.device_global_maps(self.batch, slots, pos)
        _lib.check_faults()
        for (e, a, st), gm in zip(todo, maps):
            s = self.batch.scenes[e]
            rid = s['robots'][a].get('id', '%d_%d' % (e, a))
            out = os.path.join(figures_dir, 'robot_id_{}'.format(rid))
            figures.save_state_figures(out, s['flags'], s['room_length'], s['room_width'], len(s['robots']),
                                       st if numpy else st.cpu().numpy(), gm)
            if occupancy_maps and (e, a) in occupancy_maps:
                occupancy_maps[(e, a)].save_figure(os.path.join(out, 'global-occupancy-map.png'))
        return states

    # -- reward lookups -----------------------------------------------------
    def distance_to_receptacle(self, positions, stream=None):
        """Mapper.distance_to_receptacle with use_shortest_path_partial_rewards (envs.py:2190-2194):
        positions [E][A][Q] (x, y[, z]) per robot (e.g. the cubes it just moved) -> [E][A] lists of
        Python floats, each robot's own map, the receptacle as the SPFA source.  One launch."""
        Qs = [len(p) for pe in positions for p in pe]
        Q = max(Qs) if Qs else 0
        n = self.batch.N
        tgt = np.zeros((n, max(Q, 1), 2))
        for (e, a), k in self.slot.items():
            if self.batch.scenes[e]['receptacle_position'] is None:
                raise ValueError('distance_to_receptacle needs a receptacle (not a rescue env)')
            for q, p in enumerate(positions[e][a]):
                tgt[k, q] = p[:2]
        if Q:
            # from the receptacle arrays get_state left in the cache where the maps are unchanged
            # (the reference's GridGraph cache), a full SSSP elsewhere (StateBatch.receptacle_distances)
            d = self.batch.receptacle_distances(tgt[:, :Q], stream=stream)
            if stream is not None:
                torch.cuda.current_stream(self.batch.device).wait_stream(stream)
            d = d.cpu().numpy()
            _lib.check_faults()
        else:
            d = np.zeros((n, 0))
        return [[[float(x) for x in d[self.slot[(e, a)], :len(positions[e][a])]] for a in range(len(positions[e]))]
                for e in range(self.num_envs)]

    # -- movement paths -------------------------------------------------------
    def shortest_path(self, requests, stream=None):
        """Mapper.shortest_path(source_position, target_position) (envs.py:2186-2187 ->
        OccupancyMap.shortest_path, 2478-2505), as Robot.store_new_action calls it (875-876), for a
        batch: requests [((env, robot), source_position, target_position), ...] -> one waypoint list
        per request on that robot's own map, like the reference's: the caller's source / target
        objects at the two ends (envs.py:2486, 2500-2503), (x, y, 0) tuples between.  One launch;
        a robot may appear in several requests."""
        if not requests:
            return []
        slots = [self.slot[(int(ea[0]), int(ea[1]))] for ea, _, _ in requests]
        src = np.array([[float(s[0]), float(s[1])] for _, s, _ in requests], dtype=np.float64)
        tgt = np.array([[float(t[0]), float(t[1])] for _, _, t in requests], dtype=np.float64)
        paths = self.batch.shortest_paths(src, tgt, slots=slots, stream=stream)
        for p, (_, s, t) in zip(paths, requests):
            p[0], p[-1] = s, t
        return paths


MAX_WINDOW_CELLS, MAX_WINDOW_W = 9024, 120  # SIMAPS_MAX_ROOM_CELLS / SIMAPS_MAX_ROOM_W (include/simaps.h)


def window_fits(h, w):
    """Whether an h x w window of free cells fits the LDS-resident SSSP / SPFA kernels (the rule of
    simaps_sssp_grid / simaps_grid_path); larger windows run the global-memory kernels
    (csrc/grid_large.h): same results, slower."""
    return h >= 1 and 1 <= w <= MAX_WINDOW_W and (h + 2) * ((w + 2) | 1) <= MAX_WINDOW_CELLS


class GridGraph:
    """shortest_paths.pyx GridGraph (pyx:10-167) on the device: 8-connected grid over cells with
    grid != 0, weights 1 / float32(sqrt(2)), float32 distances, unreachable -> -1.

    Results are bit-identical to the reference SPFA (the float32 fixpoint is unique, SURVEY.md
    a10).  Like _spfa_with_cache (pyx:116-119) the images are cached per source for the life of
    the graph.  Any 2-D grid, like the reference's (pyx:24-38): when the free cells span a window
    beyond the LDS-resident limits of include/simaps.h (every reference call site passes a room
    cspace, which fits), the C ABI runs the global-memory kernels instead (`large` is then True)."""

    def __init__(self, grid, device='cuda'):
        g = torch.as_tensor(np.ascontiguousarray(grid) if isinstance(grid, np.ndarray) else grid)
        if g.dim() != 2:
            raise ValueError('grid must be 2-D')
        self.device = _batch.resolve_device(device)
        self.grid = g.to(device=self.device, dtype=torch.uint8).contiguous()
        self.shape = tuple(self.grid.shape)
        free = torch.nonzero(self.grid)
        if free.numel():
            (i0, j0), (i1, j1) = free.min(0).values.tolist(), free.max(0).values.tolist()
            self.window = (i0, j0, i1 - i0 + 1, j1 - j0 + 1)
        else:
            self.window = (0, 0, 1, 1)
        self.large = not window_fits(self.window[2], self.window[3])
        self._cache = {}

    def _check_source(self, source):
        i, j = int(source[0]), int(source[1])
        if not (0 <= i < self.shape[0] and 0 <= j < self.shape[1]):
            raise IndexError('cell %s outside the %dx%d grid' % (((i, j),) + self.shape))
        return i, j

    def shortest_path_images(self, sources, stream=None):
        """Batched shortest_path_image for many sources: [len(sources), H, W] device tensor."""
        srcs = [self._check_source(s) for s in sources]
        todo = [s for s in dict.fromkeys(srcs) if s not in self._cache]
        if todo:
            grids = self.grid.unsqueeze(0).expand(len(todo), *self.shape).contiguous()
            imgs = _batch.sssp_grid(grids, torch.tensor(todo, dtype=torch.int32), window=self.window, stream=stream)
            if stream is not None:  # cached images are read on the current stream by later calls
                torch.cuda.current_stream(self.device).wait_stream(stream)
            for k, s in enumerate(todo):
                self._cache[s] = imgs[k]
        return torch.stack([self._cache[s] for s in srcs]) if srcs else \
            torch.empty((0,) + self.shape, dtype=torch.float32, device=self.device)

    def shortest_path_image(self, source):
        """(H, W) float32 NumPy image of distances from `source` (pyx:165-167)."""
        img = self.shortest_path_images([source])[0].cpu().numpy()
        _lib.check_faults()
        return img

    def shortest_path(self, source, target):
        """Waypoint cells [(i, j), ...] from `source` to `target` (pyx:121-154): the SPFA parent
        walk, approximate_polygon(tolerance=1) and line-of-sight pruning, source first."""
        return self.shortest_paths([(source, target)])[0]

    def shortest_paths(self, pairs, stream=None):
        """Batched shortest_path over (source, target) cell pairs, one launch."""
        pairs = [(self._check_source(s), self._check_source(t)) for s, t in pairs]
        if not pairs:
            return []
        grids = self.grid.unsqueeze(0).expand(len(pairs), *self.shape).contiguous()
        return _batch.grid_paths(grids, [p[0] for p in pairs], [p[1] for p in pairs], window=self.window,
                                 max_points=max(256, self.shape[0] + self.shape[1]), stream=stream, grow=True)

    def shortest_path_distance(self, source, target):
        """dists[target] from `source` as a Python float (pyx:156-163); -1 if unreachable."""
        i, j = self._check_source(target)
        return float(self.shortest_path_images([source])[0][i, j])


def _robot_type(robot):
    """'lifting_robot' ... from a type name or a reference Robot object (reference_adapter.robot_type)."""
    if isinstance(robot, str):
        if robot not in _lib.TYPE_IDS:
            raise ValueError('unknown robot type %r' % robot)
        return robot
    from .reference_adapter import robot_type
    return robot_type(robot)


class OccupancyMap:
    """envs.OccupancyMap (envs.py:2409-2524) on the device, for one robot's map.

    The reference keeps the occupancy grid of one robot, and on update() derives from it the
    configuration space (disk of the robot's radius), the EDT snap table (closest_cspace_indices),
    cspace_thin and a GridGraph; shortest_path / shortest_path_distance / shortest_path_image answer
    movement and reward queries on them.  Here the grid lives on the device and every derived map is a
    kernel output of the C ABI (simaps_occupancy_scatter, simaps_build_cspace, simaps_snap_sources,
    simaps_shortest_path, simaps_sp_distance, simaps_sssp_grid), bit for bit the reference's.
    `robot`: a reference Robot object or a type name ('lifting_robot', ...).  The NumPy views
    (occupancy_map, configuration_space, cspace_thin, closest_cspace_indices) are copies made on
    access; closest_cspace_indices (the whole [2, H, W] table) is computed on first access after an
    update.  show_map=True keeps the reference's map figure (envs.py:2434-2443, 2529-2555) for
    save_figure: the free-space map is marked on the device by the same scatter kernel, the figure is a
    headless matplotlib Figure (no window, no plt.pause)."""

    def __init__(self, robot, room_length, room_width, show_map=False, device='cuda'):
        from . import constants as K
        self.robot = robot
        self.room_length, self.room_width = room_length, room_width
        self.show_map = bool(show_map)
        typ = _robot_type(robot)
        H, W = K.padded_room_shape(room_width, room_length)
        rob = {'type': typ, 'cls': K.ROBOT_TYPES.index(typ), 'group_index': 0, 'position': (0.0, 0.0, 0.0),
               'heading': 0.0, 'lift_state': None, 'idle': True, 'waypoint_positions': None, 'waypoint_index': None,
               'target_ee': None}
        scene = {'env_name': 'occupancy_map', 'room_length': room_length, 'room_width': room_width,
                 'flags': dict(K.DEFAULT_FLAGS), 'robot_config': [{typ: 1}], 'H': H, 'W': W,
                 'receptacle_position': None, 'robots': [rob],
                 'occupancy': np.zeros((1, H, W), np.uint8), 'overhead': np.zeros((1, H, W), np.float32)}
        self._b = _batch.StateBatch([scene], device=device)
        self._cspace = self._thin = self._closest = None
        self.grid_graph = None
        if self.show_map:  # envs.py:2434-2443
            from matplotlib.figure import Figure
            self.fig_width = room_length + 2 * K.HALF_WIDTH
            self.fig_height = room_width + 2 * K.HALF_WIDTH
            self.fig = Figure(figsize=(4 * self.fig_width, 4 * self.fig_height))
            self._free = torch.zeros_like(self._b.occupancy)
            self._update_map_visualization()

    # -- the reference's attributes, as host copies ------------------------------------------------------
    @property
    def occupancy_map(self):
        return self._b.occupancy[0].cpu().numpy()

    @occupancy_map.setter
    def occupancy_map(self, grid):
        self._b.set_maps(occupancy=torch.as_tensor(np.asarray(grid, dtype=np.uint8))[None])
        self._derive()

    @property
    def configuration_space(self):
        return None if self._cspace is None else self._cspace.cpu().numpy()

    @property
    def cspace_thin(self):
        return None if self._thin is None else self._thin.cpu().numpy()

    @property
    def closest_cspace_indices(self):
        """[2, H, W] int32: scipy distance_transform_edt(1 - cspace, return_indices=True) (envs.py:2455)."""
        if self._cspace is None:
            return None
        if self._closest is None:
            H, W = self._b.H, self._b.W
            ii, jj = torch.meshgrid(torch.arange(H, dtype=torch.int32), torch.arange(W, dtype=torch.int32), indexing='ij')
            px = torch.stack([ii, jj], -1).reshape(1, H * W, 2)
            out = self._b.snap_pixels(px).cpu().numpy()
            _lib.check_faults()
            self._closest = out[0].T.reshape(2, H, W).copy()
        return self._closest

    # -- OccupancyMap.update (envs.py:2445-2466) -----------------------------------------------------------
    def update(self, points, seg, obstacle_seg_value):
        """points [..., 3] / seg [...] (Camera.capture_image, envs.py:1927-1955): the obstacle points mark
        the occupancy grid, then the cspace, cspace_thin and the grid graph are rebuilt."""
        pts = np.asarray(points, dtype=np.float32).reshape(1, -1, 3)
        sg = np.asarray(seg, dtype=np.float32).reshape(1, -1)
        self._b.scatter_obstacles(pts, sg, obstacle_seg_value)
        self._derive()
        if self.show_map:  # envs.py:2462-2466: the points that are not obstacles mark the free-space map
            v = float(obstacle_seg_value)
            d = torch.as_tensor(sg, device=self._b.device).double()
            close = (d - v).abs() <= 1e-8 + 1e-5 * abs(v)  # np.isclose in float64; NaN is never close
            self._b.scatter_obstacles(pts, (~close).float(), 1.0, out=self._free)
            self._update_map_visualization()

    @property
    def free_space_map(self):
        """show_map only: uint8 [H, W], 1 where a non-obstacle point was seen (envs.py:2442, 2463-2465)."""
        return self._free[0].cpu().numpy() if self.show_map else None

    def _update_map_visualization(self):
        """envs.py:2529-2555, drawn into the headless figure."""
        from . import constants as K
        occ = self.occupancy_map
        vis = np.zeros(occ.shape) + 0.5
        vis[self.free_space_map == 1] = 1
        vis[occ == 1] = 0
        self.fig.clf()
        self.fig.add_axes((0, 0, 1, 1))
        ax = self.fig.gca()
        ax.axis('off')
        ax.axis([-self.fig_width / 2, self.fig_width / 2, -self.fig_height / 2, self.fig_height / 2])
        height, width = vis.shape
        height, width = height / K.LOCAL_MAP_PIXELS_PER_METER, width / K.LOCAL_MAP_PIXELS_PER_METER
        ax.imshow(255.0 * vis, extent=(-width / 2, width / 2, -height / 2, height / 2), cmap='gray', vmin=0, vmax=255.0)
        wp = getattr(self.robot, 'waypoint_positions', None)
        if wp is not None:
            wp = np.array(wp)
            ax.plot(wp[:, 0], wp[:, 1], color='r', marker='.')
        ee = getattr(self.robot, 'target_end_effector_position', None)
        if ee is not None:
            ax.plot(ee[0], ee[1], color='r', marker='x')

    def _derive(self):
        cs, th = self._b.build_cspace()
        self._cspace, self._thin, self._closest = cs[0], th[0], None
        self.grid_graph = GridGraph(self._cspace, device=self._b.device)

    def _need_update(self):
        if self._cspace is None:
            raise RuntimeError('OccupancyMap: call update() first (the reference has no cspace before it)')

    def _closest_valid_cspace_indices(self, i, j):
        self._need_update()
        out = self._b.snap_pixels(torch.tensor([[[int(i), int(j)]]], dtype=torch.int32)).cpu().numpy()
        _lib.check_faults()
        return out[0, 0]

    def _pixel(self, position):
        from . import constants as K
        return K.position_to_pixel_indices(position[0], position[1], (self._b.H, self._b.W))

    # -- queries (envs.py:2478-2517) --------------------------------------------------------------------
    def shortest_path(self, source_position, target_position):
        """Waypoints [source_position, (x, y, 0), ..., target_position] (envs.py:2478-2505)."""
        self._need_update()
        path = self._b.shortest_paths(np.array([[float(source_position[0]), float(source_position[1])]]),
                                      np.array([[float(target_position[0]), float(target_position[1])]]))[0]
        path[0], path[-1] = source_position, target_position
        return path

    def shortest_path_distance(self, source_position, target_position):
        """Shortest-path length in metres (envs.py:2507-2512); -1/96 if unreachable."""
        self._need_update()
        d = self._b.shortest_path_distances(np.array([[float(source_position[0]), float(source_position[1])]]),
                                            np.array([[[float(target_position[0]), float(target_position[1])]]]))
        d = float(d.cpu().numpy()[0, 0])
        _lib.check_faults()
        return d

    def shortest_path_image(self, position):
        """[H, W] float32 image of shortest-path distances (metres) from `position`'s snapped pixel,
        -1/96 where unreachable (envs.py:2514-2517)."""
        self._need_update()
        i, j = self._closest_valid_cspace_indices(*self._pixel(position))
        return self.grid_graph.shortest_path_image((int(i), int(j))) / np.float32(96)

    def save_figure(self, output_path):
        """envs.py:2519-2521: the map figure of the last update, as the reference saves it."""
        assert self.show_map
        self.fig.savefig(output_path, bbox_inches='tight', pad_inches=0)


__all__ = ['VectorEnvObservations', 'GridGraph', 'OccupancyMap', 'robot_groups', 'window_fits']
