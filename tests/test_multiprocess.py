"""world_size-2 gloo rehearsal of bench.py's multi-GPU path on the CPU.

The path shards whole envs across ranks with no data-path collective: the only distributed
operations are the barriers around the timed region and the max-over-ranks reduction of the
timings.  These tests run exactly those helpers (bench.rank_envs / timed_steps / max_over_ranks)
under torch.distributed with the gloo backend, plus the per-rank host packing of the scene
descriptors, with a CPU stand-in for the kernel launch.
"""
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, envs_per_rank, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
    import torch.distributed as dist
    import bench
    from simaps import synthetic
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        ids = bench.rank_envs(rank, envs_per_rank)
        scenes = [synthetic.make_scene('lifting_4-small_divider', e) for e in ids]
        # Host packing happens per rank on its own shard: agent records index the rank-local envs.
        import simaps.batch as B  # noqa: F401  (needs libsimaps.so only for the dtypes' module)
        robots, envs, ag, paths = B.pack_descriptors(scenes, [(e, a) for e in range(len(scenes)) for a in range(4)])
        assert ag['env'].max() == len(scenes) - 1 and np.array_equal(ag['map_slot'], np.arange(len(ag)))
        # Rank 1 is the slow rank: the reported time must be its time on every rank.
        delay = 0.02 if rank == 1 else 0.0
        calls = []

        def step(k):
            calls.append(k)
            time.sleep(delay)

        el = bench.timed_steps(step, steps=5, warmup=2, sync=lambda: None, world=world)
        mx = bench.max_over_ranks([float(rank), -float(rank)], world)
        np.save(os.path.join(out_dir, 'r%d.npy' % rank),
                np.array([el, mx[0], mx[1], len(calls), sum(k >= 0 for k in calls), ids[0], ids[-1],
                          float(robots['x'].sum())]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_sharding_and_timing(tmp_path):
    world, E = 2, 3
    mp.spawn(_worker, args=(world, _free_port(), E, str(tmp_path)), nprocs=world, join=True)
    r = [np.load(os.path.join(tmp_path, 'r%d.npy' % k)) for k in range(world)]
    for k in range(world):
        el, mx0, mx1, ncalls, ntimed, first, last, _ = r[k]
        assert el >= 5 * 0.02 * 0.9          # the slow rank's 5 timed steps dominate on both ranks
        assert mx0 == world - 1 and mx1 == 0  # element-wise max over ranks
        assert ncalls == 7 and ntimed == 5    # exactly K timed steps after W warmup steps
        assert (first, last) == (k * E, k * E + E - 1)
    assert abs(r[0][0] - r[1][0]) < 1e-12    # one job time, identical on every rank
    assert r[0][7] != r[1][7]                # different envs (seeds) on different ranks


def test_rank_envs_partition():
    sys.path.insert(0, ROOT)
    import bench
    for world in (1, 2, 4, 8):
        ids = [e for r in range(world) for e in bench.rank_envs(r, 128)]
        assert ids == list(range(world * 128))
