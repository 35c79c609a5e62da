"""ctypes binding of libsimaps.so (the C ABI declared in include/simaps.h).

torch is imported FIRST so that libsimaps.so binds to the HIP runtime torch already loaded
(both resolve SONAME libamdhip64.so.7): one runtime instance, so torch device pointers and
streams are valid in our launches.  There is no CPU fallback: if the library is missing this
module raises at import.
"""
import ctypes
import os

import numpy as np
import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('SIMAPS_LIB', os.path.join(HERE, 'libsimaps.so'))

LIFTING, PUSHING, THROWING, RESCUE = 0, 1, 2, 3
TYPE_IDS = {'lifting_robot': LIFTING, 'pushing_robot': PUSHING, 'throwing_robot': THROWING, 'rescue_robot': RESCUE}
ENC_IDS = {'ramp': 0, 'binary': 1, 'line': 2, 'circle': 3}
ROT_IDS = {'fma': 0, 'plain': 1}  # SIMAPS_ROT_* (include/simaps.h)
MAX_ROBOTS = 8
MAX_PATH = 16

# numpy mirrors of the device structs (include/simaps.h), packed C layout
ROBOT_DTYPE = np.dtype([('x', '<f8'), ('y', '<f8'), ('heading', '<f8'), ('target_x', '<f8'), ('target_y', '<f8'),
                        ('type', '<i4'), ('group_index', '<i4'), ('lifting', '<i4'), ('idle', '<i4'),
                        ('intention_off', '<i4'), ('intention_len', '<i4'), ('history_off', '<i4'),
                        ('history_len', '<i4')], align=True)
ENV_DTYPE = np.dtype([('receptacle_x', '<f8'), ('receptacle_y', '<f8'), ('has_receptacle', '<i4'),
                      ('robot_off', '<i4'), ('num_robots', '<i4'), ('reserved', '<i4')], align=True)
ABI_VERSION = 8  # include/simaps.h SIMAPS_ABI_VERSION
MAX_MIXED = 8  # SIMAPS_MAX_MIXED
AGENT_DTYPE = np.dtype([('env', '<i4'), ('robot', '<i4'), ('map_slot', '<i4')], align=True)
assert ROBOT_DTYPE.itemsize == 72 and ENV_DTYPE.itemsize == 32 and AGENT_DTYPE.itemsize == 12


SEG_IDS_DTYPE = np.dtype([('min_obstacle', '<i4'), ('max_obstacle', '<i4'), ('receptacle', '<i4'),
                          ('min_cube', '<i4'), ('max_cube', '<i4'), ('has_receptacle', '<i4')], align=True)


class Camera(ctypes.Structure):
    """simaps_camera (include/simaps.h)."""
    _fields_ = [('height_px', ctypes.c_int32), ('width_px', ctypes.c_int32), ('near_m', ctypes.c_double),
                ('far_m', ctypes.c_double), ('cx2', ctypes.c_double), ('cy2', ctypes.c_double)]


class Config(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        'H', 'W', 'room_i0', 'room_j0', 'room_h', 'room_w', 'use_robot_map', 'use_distance_to_receptacle_map',
        'use_shortest_path_to_receptacle_map', 'use_shortest_path_map', 'use_intention_map',
        'intention_map_encoding', 'intention_map_line_thickness', 'use_history_map', 'use_intention_channels',
        'intention_channel_spatial', 'layout_chw', 'rotate_rounding')] + \
        [(n, ctypes.c_double) for n in ('distance_to_receptacle_map_scale', 'shortest_path_map_scale',
                                         'intention_map_scale', 'intention_channel_nonspatial_scale')]


class Debug(ctypes.Structure):
    """simaps_debug: optional per-agent outputs (parity tests) and the receptacle distance cache."""
    _fields_ = [('cspace', ctypes.c_void_p), ('sources', ctypes.c_void_p), ('dist', ctypes.c_void_p),
                ('status', ctypes.c_void_p), ('rec_cache', ctypes.c_void_p)]


class SimapsError(RuntimeError):
    pass


class StaleLibraryError(ImportError):
    """libsimaps.so was built from sources other than the tree's (simaps_source_hash)."""


def _check_source_hash(L, path):
    """Refuse a library built from other sources than this tree's csrc/ + include/ (a stale .so left
    over from before a kernel edit would otherwise run silently, on the GPU box too).  An A/B
    timing of another revision's build names the hash it expects in SIMAPS_AB_SOURCE_HASH."""
    from . import _srchash
    if not hasattr(L, 'simaps_source_hash'):
        if os.environ.get('SIMAPS_AB_OLD_ABI'):  # (an older revision's A/B build predates the export)
            return
        raise StaleLibraryError('%s has no simaps_source_hash: built before the stale-binary guard; rebuild it with '
                                '`make -C spatial-intention-maps_amd/csrc`' % path)
    L.simaps_source_hash.restype = ctypes.c_char_p
    built = L.simaps_source_hash().decode()
    want = os.environ.get('SIMAPS_AB_SOURCE_HASH') or _srchash.source_hash()
    if built != want:
        raise StaleLibraryError('%s was built from other sources (hash %s) than this tree\'s (%s): a stale binary -- '
                                'rebuild it with `make -C spatial-intention-maps_amd/csrc` (and `... diag` for the '
                                'diagnostic builds)' % (path, built[:16], want[:16]))


def _load(path=LIB_PATH):
    """Bind the C ABI of the library at `path` (the product libsimaps.so by default; tests also load
    diagnostic builds of the same ABI through this)."""
    if not os.path.exists(path):
        raise ImportError('libsimaps.so not found at %s -- build it with `make -C spatial-intention-maps_amd/csrc` '
                          '(or __graft_entry__.build()); there is no CPU fallback' % path)
    L = ctypes.CDLL(path)
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    L.simaps_abi_version.restype = i32
    _check_source_hash(L, path)
    L.simaps_last_error.restype = ctypes.c_char_p
    L.simaps_num_channels.argtypes = [ctypes.POINTER(Config), i32]
    L.simaps_num_channels.restype = i32
    L.simaps_pack_robots.argtypes = [i32, vp, vp, vp, vp, vp, i32, vp, vp, vp, vp]
    L.simaps_pack_robots.restype = i32
    L.simaps_robot_mask.argtypes = [i32, i32, vp]
    L.simaps_robot_mask.restype = i32
    L.simaps_get_state.argtypes = [ctypes.POINTER(Config), i32, vp, vp, vp, vp, vp, vp, vp, i32,
                                   ctypes.POINTER(Debug), vp]
    L.simaps_get_state.restype = i32
    if hasattr(L, 'simaps_get_state_mixed'):  # (ABI 8; absent only in an older revision's A/B build)
        L.simaps_get_state_mixed.argtypes = [ctypes.POINTER(Config), vp, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                             vp, vp]
        L.simaps_get_state_mixed.restype = i32
    L.simaps_sp_distance.argtypes = [ctypes.POINTER(Config), i32, vp, vp, vp, vp, vp, vp, i32, vp, vp, vp]
    L.simaps_sp_distance.restype = i32
    if hasattr(L, 'simaps_sp_lookup'):  # (ABI 7; absent only in an older revision's A/B build)
        L.simaps_rec_cache_bytes.argtypes = [ctypes.POINTER(Config)]
        L.simaps_rec_cache_bytes.restype = i32
        L.simaps_sp_lookup.argtypes = [ctypes.POINTER(Config), i32, vp, vp, vp, i32, vp, vp]
        L.simaps_sp_lookup.restype = i32
    L.simaps_shortest_path.argtypes = [ctypes.POINTER(Config), i32, vp, vp, vp, vp, vp, vp, i32, vp, vp, vp]
    L.simaps_shortest_path.restype = i32
    L.simaps_ingest.argtypes = [ctypes.POINTER(Config), ctypes.POINTER(Camera), i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp]
    L.simaps_ingest.restype = i32
    L.simaps_path_mode.argtypes = [i32]
    L.simaps_path_mode.restype = i32
    L.simaps_ingest_chunks.argtypes = [i32, i32]
    L.simaps_ingest_chunks.restype = i32
    L.simaps_sssp_grid.argtypes = [i32, i32, i32, vp, vp, vp, i32, i32, i32, i32, vp]
    L.simaps_sssp_grid.restype = i32
    L.simaps_grid_path.argtypes = [i32, i32, i32, vp, vp, vp, i32, i32, i32, i32, i32, vp, vp, vp]
    L.simaps_grid_path.restype = i32
    L.simaps_fault_status.argtypes = [i32]
    L.simaps_fault_status.restype = i32
    if hasattr(L, 'simaps_build_cspace'):  # (round 6; absent only in an older revision's A/B build)
        L.simaps_occupancy_scatter.argtypes = [ctypes.POINTER(Config), i32, vp, vp, vp, i32, ctypes.c_double, vp, vp]
        L.simaps_occupancy_scatter.restype = i32
        L.simaps_build_cspace.argtypes = [ctypes.POINTER(Config), i32, vp, vp, vp, vp, vp, vp, vp]
        L.simaps_build_cspace.restype = i32
        L.simaps_snap_sources.argtypes = [ctypes.POINTER(Config), i32, vp, vp, vp, vp, vp, i32, vp, vp]
        L.simaps_snap_sources.restype = i32
        L.simaps_global_maps.argtypes = [ctypes.POINTER(Config), i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.simaps_global_maps.restype = i32
    v = L.simaps_abi_version()
    if v != ABI_VERSION:
        if os.environ.get('SIMAPS_AB_OLD_ABI') != str(v):
            raise ImportError('libsimaps ABI version mismatch: %s has %d, this binding is %d' % (path, v, ABI_VERSION))
        # SIMAPS_AB_OLD_ABI=<n>: tools/ab_bench.sh timing an older revision's get_state, whose
        # signature is unchanged.  Only the entry points a bench render needs stay callable; any other
        # raises instead of being called with this revision's argument list.
        return _OldAbi(L, v)
    return L


class _OldAbi:
    """An older revision's library bound for an A/B timing only (see _load)."""
    ALLOWED = ('simaps_abi_version', 'simaps_last_error', 'simaps_fault_status', 'simaps_num_channels',
               'simaps_get_state')

    def __init__(self, L, version):
        self._L, self._v = L, version

    def __getattr__(self, name):
        if name in self.ALLOWED:
            return getattr(self._L, name)
        raise SimapsError('%s is not callable on the ABI-%d library loaded for an A/B timing (SIMAPS_AB_OLD_ABI); '
                          'only %s are' % (name, self._v, ', '.join(self.ALLOWED)))


lib = _load()

EXPORTED = ('simaps_abi_version', 'simaps_last_error', 'simaps_fault_status', 'simaps_num_channels',
            'simaps_robot_mask', 'simaps_pack_robots', 'simaps_get_state', 'simaps_sp_distance', 'simaps_shortest_path', 'simaps_ingest', 'simaps_ingest_chunks', 'simaps_path_mode',
            'simaps_sssp_grid', 'simaps_grid_path', 'simaps_rec_cache_bytes', 'simaps_sp_lookup',
            'simaps_get_state_mixed', 'simaps_source_hash', 'simaps_occupancy_scatter', 'simaps_build_cspace',
            'simaps_snap_sources', 'simaps_global_maps')

# error codes and device fault bits (include/simaps.h)
EINVAL, EUNSUPPORTED, EHIP, EDEVICE = -1, -2, -3, -4
FAULT_TIMEOUT, FAULT_ROUNDS, FAULT_DESCRIPTOR = 1, 2, 4


class DeviceFault(SimapsError):
    """A kernel reported SIMAPS_FAULT_* bits: the outputs of that launch are invalid."""


def check(rc, L=None):
    if rc != 0:
        L = L or lib
        cls = DeviceFault if rc == EDEVICE else SimapsError
        raise cls('libsimaps error %d: %s' % (rc, L.simaps_last_error().decode()))


def check_faults(L=None):
    """Raise DeviceFault if a completed launch reported a device-side fault (clears the word).
    Call after the stream has been synchronised (e.g. after a device->host copy of the results)."""
    L = L or lib
    f = L.simaps_fault_status(1)
    if f < 0:
        check(f, L)
    if f:
        raise DeviceFault('device fault bits 0x%x (%s): the outputs of a completed launch are invalid' % (
            f, ' '.join(n for b, n in ((FAULT_TIMEOUT, 'barrier-timeout'), (FAULT_ROUNDS, 'sssp-round-cap'),
                                       (FAULT_DESCRIPTOR, 'descriptor-clamped')) if f & b)))


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def robot_mask(robot_type, with_cube=False):
    out = np.zeros((96, 96), dtype=np.float32)
    check(lib.simaps_robot_mask(TYPE_IDS.get(robot_type, robot_type), int(with_cube), out.ctypes.data))
    return out
