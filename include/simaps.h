/* simaps.h -- C ABI of libsimaps.so, the MI355X-native observation-map pipeline of
 * Spatial Intention Maps (reference: mushroonhead/spatial-intention-maps, envs.py + shortest_paths/).
 *
 * Plain C: pointers, sizes, POD structs; no torch/HIP types in any signature.  Device pointers
 * are HIP device allocations (e.g. torch CUDA/ROCm tensors' data_ptr()).  `stream` is a
 * hipStream_t passed as void* (NULL = default stream); every compute call is asynchronous on it.
 * Return value: 0 = ok, negative = error (see SIMAPS_E*; simaps_last_error() has the text).
 * No exceptions cross the ABI.  Thread-safe: no global mutable state besides the last-error
 * string (thread-local) and the process-wide device fault word (simaps_fault_status).
 *
 * Reference interfaces replaced (file:line relative to the reference repo root):
 *   simaps_get_state    <- Mapper.get_state (envs.py:2068-2185) for a batch of agents, including
 *                          the OccupancyMap.update work it needs (envs.py:2445-2460: cspace,
 *                          EDT snap, GridGraph) minus the camera-point scatter; what
 *                          VectorEnv.get_state(all_robots=True) (envs.py:322-323) returns.
 *   simaps_sssp_grid    <- GridGraph(grid).shortest_path_image(source)
 *                          (shortest_paths/shortest_paths.pyx:24-67, 69-119, 165-167), batched.
 *   simaps_grid_path    <- GridGraph(grid).shortest_path(source, target) (shortest_paths.pyx:121-154),
 *                          batched, exact SPFA parents.
 *   simaps_sp_distance  <- OccupancyMap.shortest_path_distance (envs.py:2507-2512), i.e. the reward
 *                          lookup Mapper.distance_to_receptacle (envs.py:2190-2194) used by the
 *                          partial rewards (envs.py:1083-1088, 1211-1216, 1332-1336), batched.
 *   simaps_shortest_path <- OccupancyMap.shortest_path (envs.py:2478-2505) + GridGraph.shortest_path
 *                          (shortest_paths.pyx:121-154): the movement path of Robot.store_new_action
 *                          (envs.py:875-876), batched, exact SPFA parents.
 *   simaps_ingest       <- Robot.update_map minus the simulator: Camera.capture_image on a given depth /
 *                          segmentation frame (envs.py:1927-1955), Mapper.update (2056-2062) and the
 *                          obstacle scatter of OccupancyMap.update (2447-2450), in place, batched.
 *   simaps_robot_mask   <- Mapper._create_robot_mask (envs.py:2218-2242) (host helper).
 *   simaps_num_channels <- the channel list of Mapper.get_state (envs.py:2071-2113).
 *   simaps_get_state_mixed <- simaps_get_state over agents of several configurations, one launch.
 */
#ifndef SIMAPS_H
#define SIMAPS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SIMAPS_ABI_VERSION 8

/* error codes */
#define SIMAPS_OK 0
#define SIMAPS_EINVAL -1      /* bad argument / shape / flag combination */
#define SIMAPS_EUNSUPPORTED -2 /* valid for the reference but outside this build's limits */
#define SIMAPS_EHIP -3        /* HIP runtime error (launch / memory) */
#define SIMAPS_EDEVICE -4     /* an earlier launch reported a device-side fault (simaps_fault_status) */

/* Device-side fault bits (simaps_fault_status).  Every kernel of this library ORs them into one
 * process-wide host-mapped word when a workgroup hits a condition that makes its output invalid;
 * never set in a correct run.  The next simaps_get_state / simaps_sp_distance /
 * simaps_shortest_path / simaps_sssp_grid call returns SIMAPS_EDEVICE (and clears the word) if it
 * is set, so a fault surfaces even when no debug buffers were passed. */
#define SIMAPS_FAULT_TIMEOUT 1u    /* a wave-group barrier or scratch hand-over gave up waiting (~0.1 s) */
#define SIMAPS_FAULT_ROUNDS 2u     /* the SSSP round cap was hit (no convergence) */
#define SIMAPS_FAULT_DESCRIPTOR 4u /* a descriptor field outside this build's limits was clamped: num_robots
                                      > SIMAPS_MAX_ROBOTS, robot index >= num_robots, an env's num_robots
                                      other than num_robots_per_env with intention channels on, a used
                                      intention / history path longer than SIMAPS_MAX_PATH points; or (mixed
                                      launch) a configuration index outside [0, n_cfgs): reported, and
                                      that agent's stack is left unwritten */

/* robot classes (envs.py: LiftingRobot 1169, PushingRobot 1059, ThrowingRobot 1279, RescueRobot 1346) */
#define SIMAPS_LIFTING 0
#define SIMAPS_PUSHING 1
#define SIMAPS_THROWING 2
#define SIMAPS_RESCUE 3

/* intention_map_encoding (envs.py:2308-2340) */
#define SIMAPS_ENC_RAMP 0
#define SIMAPS_ENC_BINARY 1
#define SIMAPS_ENC_LINE 2
#define SIMAPS_ENC_CIRCLE 3

/* rotate_rounding: scipy.ndimage.rotate (envs.py:2206, 2267) computes out_center = M @ ((S-1)/2)
 * through numpy matmul -> BLAS dgemv, whose rounding depends on the numpy/OpenBLAS build and the host
 * CPU: fma(M[r][0], a0, M[r][1] * a1) on some (numpy 2.2 here, the round-1 builder host), the plain
 * M[r][0] * a0 + M[r][1] * a1 on others (numpy 1.26.4 / OpenBLAS 0.3.23 on an AVX-512 Xeon).  About
 * 4 % of headings give a different sample grid.  Pick the form of the host the reference runs on
 * (simaps.constants.host_rotate_rounding() measures it). */
#define SIMAPS_ROT_FMA 0
#define SIMAPS_ROT_PLAIN 1

/* limits of this build */
#define SIMAPS_MAX_ROBOTS 8      /* robots per env */
#define SIMAPS_MAX_PATH 16       /* points per intention / history path */
#define SIMAPS_MAX_ROOM_CELLS 9024 /* (room_h + 2) * ((room_w + 2) | 1) */
#define SIMAPS_MAX_ROOM_W 120

/* One robot of an env, as the observation path reads it (Robot / RobotController state). */
typedef struct simaps_robot {
    double x, y;            /* robot.get_position()[:2]                         (envs.py:942)  */
    double heading;         /* robot.get_heading()                              (envs.py:950)  */
    double target_x;        /* robot.target_end_effector_position[:2]           (envs.py:870)  */
    double target_y;
    int32_t type;           /* SIMAPS_LIFTING ... SIMAPS_RESCUE                                */
    int32_t group_index;    /* robot.group_index (seg value (g+5)/8, envs.py:2257)             */
    int32_t lifting;        /* LiftingRobot.lift_state == 'lifting' (envs.py:2260)             */
    int32_t idle;           /* robot.is_idle() (envs.py:937)                                   */
    int32_t intention_off;  /* RobotController.get_intention_path() (envs.py:1475) in paths[]  */
    int32_t intention_len;
    int32_t history_off;    /* get_history_path()[::-1] (envs.py:1478, 2318), ALREADY reversed */
    int32_t history_len;
} simaps_robot;

/* One env (VectorEnv) of the batch. */
typedef struct simaps_env {
    double receptacle_x, receptacle_y; /* VectorEnv.receptacle_position (envs.py:150-151) */
    int32_t has_receptacle;
    int32_t robot_off;                 /* first robot of this env in robots[] */
    int32_t num_robots;
    int32_t reserved;
} simaps_env;

/* One agent-state stack to render: robot `robot` of env `env`, whose persistent per-agent maps
 * (occupancy / overhead, the robot's own Mapper state) are slot `map_slot` of the map arrays.
 * Output stack n of a call belongs to agents[n]; rendering a subset (the robots awaiting a new
 * action, envs.py:322-323) is a shorter agents[] over the same map arrays. */
typedef struct simaps_agent {
    int32_t env;
    int32_t robot;
    int32_t map_slot;
} simaps_agent;

/* Batch-wide configuration: VectorEnv state-representation flags (envs.py:39-45) + grid. */
typedef struct simaps_config {
    int32_t H, W;                   /* Mapper.create_padded_room_zeros shape (envs.py:2384-2389) */
    int32_t room_i0, room_j0;       /* OccupancyMap._create_room_mask rect (envs.py:2468-2476)   */
    int32_t room_h, room_w;
    int32_t use_robot_map;
    int32_t use_distance_to_receptacle_map;
    int32_t use_shortest_path_to_receptacle_map;
    int32_t use_shortest_path_map;
    int32_t use_intention_map;
    int32_t intention_map_encoding; /* SIMAPS_ENC_* */
    int32_t intention_map_line_thickness;
    int32_t use_history_map;
    int32_t use_intention_channels;
    int32_t intention_channel_spatial; /* 1 = 'spatial', 0 = 'nonspatial' */
    int32_t layout_chw;             /* 0: state is [N,96,96,C] (reference HWC), 1: [N,C,96,96] */
    int32_t rotate_rounding;        /* SIMAPS_ROT_*: how the host BLAS rounds scipy.ndimage.rotate's out_center */
    double distance_to_receptacle_map_scale;
    double shortest_path_map_scale;
    double intention_map_scale;
    double intention_channel_nonspatial_scale;
} simaps_config;

/* A robot camera (Camera subclasses, envs.py:1876-2008): image size and projection constants. */
typedef struct simaps_camera {
    int32_t height_px, width_px; /* int(1.63 * 96), int(ASPECT * height) (envs.py:1895-1896) */
    double near_m, far_m;        /* Camera.NEAR, Camera.FAR */
    double cx2, cy2;             /* 2 * limit_x, 2 * limit_y, limit_y = tan(radians(FOV / 2)) (1944-1947) */
} simaps_camera;

/* Segmentation body ids of one env (Camera._ensure_initialized, envs.py:1907-1917). */
typedef struct simaps_seg_ids {
    int32_t min_obstacle, max_obstacle, receptacle, min_cube, max_cube;
    int32_t has_receptacle;      /* receptacle_id is not None */
} simaps_seg_ids;

/* Optional per-agent intermediates (device pointers, any may be NULL), for parity tests. */
typedef struct simaps_debug {
    uint8_t *cspace;   /* [N, room_h, room_w] OccupancyMap.configuration_space inside the room rect */
    int32_t *sources;  /* [N, 2, 4]: (pi, pj, snapped_i, snapped_j) for receptacle / robot sources */
    float *dist;       /* [N, 2, room_h, room_w] raw GridGraph.shortest_path_image (-1 unreachable) */
    int32_t *status;   /* [N] bit0: no free cell (sp channels undefined in the reference); bit1: SSSP
                        round cap hit (bug guard); bit2: barrier timeout; bit3: descriptor clamped;
                        bits 8+: SSSP rounds to convergence */
    void *rec_cache;   /* NOT a debug output: with use_shortest_path_to_receptacle_map, each rendered
                        agent's converged receptacle distance array is kept in its map slot's record
                        (simaps_rec_cache_bytes(cfg) bytes per slot, slot agents[n].map_slot) for
                        simaps_sp_lookup -- the reference's GridGraph cache that get_state fills for
                        Mapper.distance_to_receptacle (envs.py:2189-2194, shortest_paths.pyx:116-119,
                        156-163).  Valid until the slot's occupancy map changes; the caller tracks that. */
} simaps_debug;

int simaps_abi_version(void);
const char *simaps_last_error(void);
/* sha256 (hex) of the sources this library was built from (the .hip / .h / .inc files of csrc/ and this header, as
 * simaps/_srchash.py computes it; "unknown" if built without it).  No reference counterpart: the
 * reference rebuilds its Cython extension from source (shortest_paths/setup.py:1-6); the Python
 * binding refuses a library whose hash differs from the tree's, i.e. a stale binary. */
const char *simaps_source_hash(void);

/* The device-side fault word (SIMAPS_FAULT_* bits) as of the launches that have completed: call
 * after synchronising the stream to cover a given launch.  clear != 0 resets it.  Returns the bits
 * (>= 0) or SIMAPS_EHIP if the host-mapped word could not be allocated. */
int simaps_fault_status(int clear);

/* Number of channels C of the stack for an env with `num_robots` robots (envs.py:2071-2113). */
int simaps_num_channels(const simaps_config *cfg, int num_robots);

/* Host helper: the per-step robot descriptors from arrays (the drop-in's array fast path), HOST memory.
 *   pose [R][3] (x, y, heading), target [R][2] (target_end_effector_position[:2]), flags [R] (bit 0
 *   idle, bit 1 LiftingRobot lift_state == 'lifting'), type_group [R][2] (SIMAPS_* class, group_index),
 *   waypoints [R][K][2] (robot.waypoint_positions[:, :2], padded), wp_count [R] (len(waypoint_positions),
 *   -1 = None: a robot that has not acted yet, which must be idle), wp_index [R]
 *   (controller.waypoint_index) -> robots [R] and paths [R][2 * SIMAPS_MAX_PATH][2]: robot r's
 *   intention path (RobotController.get_intention_path, envs.py:1475-1476) at point 2 r P, its reversed
 *   history path (get_history_path()[::-1], envs.py:1478-1479, 2318) at 2 r P + P (P = SIMAPS_MAX_PATH).
 *   Byte-identical to packing the same robots one by one.  SIMAPS_EUNSUPPORTED if a path exceeds P points. */
int simaps_pack_robots(int R, const double *pose, const double *target, const int32_t *flags, const int32_t *type_group,
                       const double *waypoints, int K, const int32_t *wp_count, const int32_t *wp_index,
                       simaps_robot *robots, double *paths);

/* Host helper: Mapper._create_robot_mask(cls, show_lifted_cube) into out[96*96] (float32, host). */
int simaps_robot_mask(int type, int with_cube, float *out);

/* Batched Mapper.get_state (+ the OccupancyMap.update work it needs).
 *   agents[N], envs[E], robots[R], paths[P][2] (fp64 x, y), all DEVICE pointers;
 *   occupancy [M, H, W] uint8 and overhead [M, H, W] float32: the per-agent global maps
 *   (OccupancyMap.occupancy_map, Mapper.global_overhead_map_without_robots), DEVICE, indexed by
 *   agents[n].map_slot (M = number of map slots, any N <= M of them rendered per call);
 *   state: [N, 96, 96, C] (or [N, C, 96, 96] if cfg->layout_chw) float32, DEVICE, C =
 *   simaps_num_channels(cfg, num_robots) -- every env of one call must have the same robot count
 *   when intention channels are on.  `num_robots_per_env` is that count (or 0 if unused); an env
 *   with another count is clamped to it and reported (SIMAPS_FAULT_DESCRIPTOR), never written past
 *   its agents' stacks.  dbg may be NULL. */
int simaps_get_state(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                     const simaps_robot *robots, const double *paths, const uint8_t *occupancy,
                     const float *overhead, float *state, int num_robots_per_env, const simaps_debug *dbg,
                     void *stream);

/* simaps_get_state over agents of up to SIMAPS_MAX_MIXED configurations in ONE launch (the
 * reference's multiprocess collector runs all its workers on one configuration,
 * train_multiprocess.py:159-166, 217-228; collectors of different configurations then share a
 * launch).  cfgs[n_cfgs] and num_robots_per_env[n_cfgs] are HOST
 * arrays (copied into the launch); everything else is DEVICE:
 *   agent_cfg [N] int32   the configuration of agent n (index into cfgs)
 *   map_off   [M] int64   element offset of map slot m in occupancy / overhead (its maps are
 *                         H x W of its agents' configuration; slots of one configuration may be packed
 *                         back to back after those of another)
 *   out_off   [N] int64   float offset of agent n's stack in state (96 * 96 * C of its configuration,
 *                         in its configuration's layout)
 * agents / envs / robots / paths as for simaps_get_state (one combined descriptor for all envs).
 * With intention channels, num_robots_per_env[k] is the robot count of every env of entry k (two
 * robot counts of one configuration are two entries).  Bit-identical to one simaps_get_state launch
 * per configuration.  No debug outputs or receptacle cache.  The offsets are the caller's: they are
 * not range-checked on the device (an agent_cfg outside [0, n_cfgs) is reported,
 * SIMAPS_FAULT_DESCRIPTOR, and that agent's stack is not written).  SIMAPS_EINVAL for n_cfgs outside [1, SIMAPS_MAX_MIXED] or a bad
 * configuration. */
#define SIMAPS_MAX_MIXED 8
int simaps_get_state_mixed(const simaps_config *cfgs, const int32_t *num_robots_per_env, int n_cfgs, int N,
                           const simaps_agent *agents, const int32_t *agent_cfg, const simaps_env *envs,
                           const simaps_robot *robots, const double *paths, const uint8_t *occupancy,
                           const int64_t *map_off, const float *overhead, float *state, const int64_t *out_off,
                           void *stream);

/* Batched OccupancyMap.shortest_path_distance(source_position, target_position) / 96 (Python float
 * semantics: the float32 SPFA distance converted to double, divided by 96.0; unreachable -> -1 / 96):
 *   on agent n's own map (occupancy slot agents[n].map_slot, its robot class's cspace radius),
 *   sources [N][2] and targets [N][Q][2] are fp64 (x, y) positions, out [N][Q] fp64, all DEVICE.
 *   Both ends are snapped to the nearest free cspace cell exactly like the reference (scipy EDT). */
int simaps_sp_distance(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                       const simaps_robot *robots, const uint8_t *occupancy, const double *sources,
                       const double *targets, int Q, double *out, void *rec_cache, void *stream);
/*   rec_cache (may be NULL): as simaps_debug.rec_cache -- when every source is its env's receptacle
 *   position, each agent's distance array from it is also kept in its map slot's record, so later
 *   lookups from the receptacle can use simaps_sp_lookup (the cache of the reference's
 *   GridGraph._spfa_with_cache, shortest_paths.pyx:116-119). */

/* Bytes of one map slot's record in a receptacle distance cache (simaps_debug.rec_cache): a 16-byte
 * header and the room rect's (room_h + 2) x ((room_w + 2) | 1) float32 distance array. */
int simaps_rec_cache_bytes(const simaps_config *cfg);

/* Mapper.distance_to_receptacle (envs.py:2190-2194, shortest-path partial rewards) answered from the
 * cache, as the reference answers it from the GridGraph that get_state filled: per agent n, the
 *   record of slot agents[n].map_slot (written by simaps_get_state / simaps_sp_distance for the
 *   slot's current map), targets [N][Q][2] fp64 (x, y), out [N][Q] fp64 -- the same values as
 *   simaps_sp_distance with the receptacle as the source: each target snapped to its nearest free
 *   cspace cell (scipy EDT, rebuilt from the cached array only for targets on blocked pixels), the
 *   float32 distance / 96, unreachable -> -1 / 96.  All DEVICE.  A record of another map is not
 *   detected: the caller keeps the cache in step with the maps. */
int simaps_sp_lookup(const simaps_config *cfg, int N, const simaps_agent *agents, const void *rec_cache,
                     const double *targets, int Q, double *out, void *stream);

/* Batched OccupancyMap.shortest_path(source_position, target_position) on agent n's own map:
 *   sources [N][2], targets [N][2] fp64 (x, y); out_xy [N][max_points][2] fp64 waypoints (first =
 *   source, last = target, as the reference returns them), out_count [N] = number of waypoints, or
 *   -needed if max_points is too small.  All DEVICE.  The SPFA runs exactly like pyx:69-114 (edge
 *   order, SLF swap), so the parents -- and hence the waypoints -- are the reference's. */
int simaps_shortest_path(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                         const simaps_robot *robots, const uint8_t *occupancy, const double *sources,
                         const double *targets, int max_points, double *out_xy, int32_t *out_count, void *stream);

/* Which path kernels simaps_shortest_path / simaps_grid_path launch (host-side, process-wide; returns
 * the previous mode): 1 compact (the SPFA runs to an empty queue); 2 early exit (the SSSP fixpoint
 * by directional sweeps first, then the SPFA only until every vertex of the target's parent chain
 * has its final distance -- whose parent then can no longer change; the fixpoint is parked in device
 * scratch taken from the default memory pool in stream order on the launch stream and returned right
 * after the launch -- a launch being captured into a graph takes the compact kernels instead);
 * 3 early exit with the sweeps overlapped (they run beside the SPFA in the same workgroup, the
 * fixpoint in LDS: no scratch, graph capture keeps it; half the queries per CU of mode 2);
 * 0 automatic: 3 while the whole launch is resident at once at mode 3's residency (N <= CUs x 2
 * small-room / x 1 large-room queries), else 2.  Modes 0-3 return the reference's waypoints
 * exactly.  (Round 6 measured an opt-in parent rule on the SSSP fixpoint instead of the SPFA:
 * 3-13x faster, but 88.7 % of fuzz paths within demo.py's atol=2 against a 99.9 % bar -- not kept,
 * DESIGN.md section 9.) */
int simaps_path_mode(int mode);

/* Batched observation ingest into the per-agent maps (occupancy / overhead [M, H, W], slot
 *   agents[n].map_slot), from depth [N][Hc][Wc] float32 (pybullet depth buffer) and seg_raw
 *   [N][Hc][Wc] int32 (body ids), cam_params [N][9] fp64 = _get_camera_params(robot pose)
 *   (position, target, up; envs.py:1962-2008), seg_ids [E] per env.  keys: uint64 [M, H, W]
 *   scratch tagged with `epoch`: all zero before the first launch, then never cleared by the
 *   library -- each launch passes an epoch in [1, 255] larger than every earlier launch's on this
 *   key map since it was last zeroed (when the epoch would wrap, zero the key map and restart at
 *   1).  epoch 0 is the zeroing mode: the key map must be all zero on entry, and the launch zeroes
 *   every key it wrote before it ends (one store per touched key more), so it is all zero on exit
 *   -- the only mode allowed while `stream` is being captured into a graph, whose replays all
 *   reuse the captured epoch; boxes: uint32 [N, simaps_ingest_chunks(Hc, Wc), 4] scratch (any
 *   contents).  The frames'
 *   map slots must be distinct.  All DEVICE.  Points with equal z on one pixel: the later camera
 *   pixel wins (the reference's np.argsort leaves that order unspecified).
 *   SIMAPS_EINVAL: epoch outside [0, 255].
 *   SIMAPS_EUNSUPPORTED: camera width outside [67, 1024], Hc * Wc >= 2^20, N > 65535, or an epoch
 *   other than 0 while `stream` is capturing
 *   (two launches on `stream`: a point pass over chunks of 2048 camera pixels with per-chunk LDS
 *   max-reduction that also records each chunk's box of touched map pixels, then one sweep of each
 *   frame's box). */

/* Point-pass chunks (2048 camera pixels each) per frame of an Hc x Wc camera: the boxes scratch of
 *   simaps_ingest holds 4 uint32 per chunk and frame.  SIMAPS_EINVAL for a non-positive size. */
int simaps_ingest_chunks(int height_px, int width_px);

int simaps_ingest(const simaps_config *cfg, const simaps_camera *cam, int N, const simaps_agent *agents,
                  const simaps_seg_ids *seg_ids, const double *cam_params, const float *depth, const int32_t *seg_raw,
                  float *overhead, uint8_t *occupancy, uint64_t *keys, uint32_t *boxes, int epoch, void *stream);

/* Batched GridGraph(grid).shortest_path_image(source):
 *   grids [B, H, W] uint8 (nonzero = free), sources [B, 2] int32 (row, col), out dists [B, H, W]
 *   float32 (-1 unreachable, like pyx:110-112), all DEVICE.  All free cells of every grid must lie
 *   in the window rows [wi0, wi0+wh) x cols [wj0, wj0+ww) (cells outside it are treated as blocked).
 *   A window with (wh+2)*((ww+2)|1) <= SIMAPS_MAX_ROOM_CELLS and ww <= SIMAPS_MAX_ROOM_W runs the
 *   LDS-resident kernel; any larger one the global-memory kernels: the tiled fixpoint (62 x 62-cell
 *   tiles through LDS from a queue of dirty tiles) up to 4,096 tiles, the whole-window sweeps beyond
 *   (same results; scratch from the library's stream-ordered pool, so SIMAPS_EUNSUPPORTED while
 *   `stream` is being captured). */
int simaps_sssp_grid(int B, int H, int W, const uint8_t *grids, const int32_t *sources, float *dists,
                     int wi0, int wj0, int wh, int ww, void *stream);

/* Batched GridGraph(grid).shortest_path(source, target) (shortest_paths.pyx:121-154) on raw cells:
 *   grids [B, H, W] uint8 (nonzero = free), sources / targets [B, 2] int32 (row, col); out_ij
 *   [B][max_points][2] int32 waypoint cells (source first, like pyx:152's reversed list), out_count
 *   [B] = number of waypoints, or -needed if max_points is too small.  All DEVICE.  The SPFA replays
 *   pyx:69-114 (edge order, SLF swap), so parents -- and waypoints -- are the reference's; the
 *   line-of-sight pruning counts cells with grid != 1 as blocked (uint8 `1 - grid`, pyx:146).  The
 *   window rule of simaps_sssp_grid applies (larger windows: the global-memory fixpoint, then one
 *   wave per query replays the SPFA).  An unreachable target gives [target] (pyx:136-137). */
int simaps_grid_path(int B, int H, int W, const uint8_t *grids, const int32_t *sources, const int32_t *targets,
                     int wi0, int wj0, int wh, int ww, int max_points, int32_t *out_ij, int32_t *out_count,
                     void *stream);

/* ---- OccupancyMap (envs.py:2409-2524) as its own drop-in (round 6) ----------------------------------
 * The per-agent maps of simaps_get_state / simaps_ingest ([M, H, W], slot agents[n].map_slot), with the
 * agent's robot class (envs / robots records as for simaps_get_state) choosing the cspace disk.  All
 * buffers DEVICE. */

/* OccupancyMap.update's obstacle scatter (envs.py:2445-2450) from a point cloud: for agent n, points
 *   [N][P][3] float32 (x, y, z) and seg [N][P] float32 (Camera.capture_image's outputs, flattened);
 *   every point with np.isclose(seg, obstacle_seg_value) (|seg - v| <= 1e-8 + 1e-5 |v|, float64) sets
 *   occupancy[slot][i][j] = 1 at Mapper.position_to_pixel_indices(x, y) (envs.py:2391-2397, float32,
 *   clipped).  Points are never removed (the reference only ever sets obstacles). */
int simaps_occupancy_scatter(const simaps_config *cfg, int N, const simaps_agent *agents, const float *points,
                             const float *seg, int P, double obstacle_seg_value, uint8_t *occupancy, void *stream);

/* The maps OccupancyMap.update derives (envs.py:2453-2456), over the whole grid, per agent n:
 *   cspace [N][H][W] u8 = configuration_space: 1 - max(1 - room_mask, binary_dilation(occupancy,
 *   disk(floor(RADIUS * 96)))) -- 1 = free, 0 outside the room rect;
 *   cspace_thin [N][H][W] u8 = 1 - binary_dilation(min(room_mask, occupancy), disk(3)).
 *   Either may be NULL (not both).  Replaces reading om.configuration_space / om.cspace_thin. */
int simaps_build_cspace(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                        const simaps_robot *robots, const uint8_t *occupancy, uint8_t *cspace, uint8_t *cspace_thin,
                        void *stream);

/* OccupancyMap._closest_valid_cspace_indices (envs.py:2523-2524) = closest_cspace_indices[:, i, j], the
 *   scipy distance_transform_edt(1 - cspace, return_indices=True) feature transform (its tie rule) at
 *   query pixels: pixels [N][Q][2] int32 (i, j) -> out [N][Q][2] int32 (snapped i, j).  A free pixel is
 *   itself.  A pixel outside the grid, or a map without any free cell, gives (-1, -1) (numpy would
 *   wrap negative indices / return scipy's value for an all-background image). */
int simaps_snap_sources(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                        const simaps_robot *robots, const uint8_t *occupancy, const int32_t *pixels, int Q,
                        int32_t *out, void *stream);

/* The global maps of Mapper.get_state(save_figures=True) (envs.py:2115-2182), per agent n over the whole
 * grid, [N][H][W] float32 each (any may be NULL; DEVICE): overhead_map = _create_global_overhead_map
 * (2244-2249), robot_map = _create_global_robot_map(seg=False) (2251-2276), history_map / intention_map =
 * _create_global_intention_or_history_map('history' / the configuration's encoding) (2302-2347).
 * Descriptors as for simaps_get_state (overhead [M][H][W]: the maps without robots, slot
 * agents[n].map_slot).  A debug export (the fused kernel keeps only each agent's 136 x 136 crop); the
 * shortest-path maps come from simaps_build_cspace + simaps_snap_sources + simaps_sssp_grid. */
int simaps_global_maps(const simaps_config *cfg, int N, const simaps_agent *agents, const simaps_env *envs,
                       const simaps_robot *robots, const double *paths, const float *overhead, float *overhead_map,
                       float *robot_map, float *history_map, float *intention_map, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SIMAPS_H */
