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

        own = []
        el = bench.timed_steps(step, steps=5, warmup=2, sync=lambda: None, world=world, own=own)
        mx = bench.max_over_ranks([float(rank), -float(rank)], world)
        # the bench line's per-rank report: all-gathered rows + the group's view
        row = dict(bench.device_identity('cpu'), rank=rank, local_rank=rank, host='h', env_range=[ids[0], ids[-1]],
                   stacks_per_step=4 * len(ids), steps=5, seconds=own[0], kernel_ms=0.0, pci='cpu-rank%d' % rank)
        rep = bench.rank_report(row, world)
        import json
        with open(os.path.join(out_dir, 'rep%d.json' % rank), 'w') as f:
            json.dump(rep, f)
        np.save(os.path.join(out_dir, 'r%d.npy' % rank),
                np.array([el, mx[0], mx[1], len(calls), sum(k >= 0 for k in calls), ids[0], ids[-1],
                          float(robots['x'].sum()), own[0]]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_sharding_and_timing(tmp_path):
    world, E = 2, 3
    mp.spawn(_worker, args=(world, _free_port(), E, str(tmp_path)), nprocs=world, join=True)
    r = [np.load(os.path.join(tmp_path, 'r%d.npy' % k)) for k in range(world)]
    for k in range(world):
        el, mx0, mx1, ncalls, ntimed, first, last, _, _ = r[k]
        assert el >= 5 * 0.02 * 0.9          # the slow rank's 5 timed steps dominate on both ranks
        assert mx0 == world - 1 and mx1 == 0  # element-wise max over ranks
        assert ncalls == 7 and ntimed == 5    # exactly K timed steps after W warmup steps
        assert (first, last) == (k * E, k * E + E - 1)
    assert abs(r[0][0] - r[1][0]) < 1e-12    # one job time, identical on every rank
    assert r[0][7] != r[1][7]                # different envs (seeds) on different ranks
    # the job time runs from the earliest rank's start to the latest rank's end: at
    # least every rank's own time, and here only the barrier-exit skew more
    assert max(r[0][8], r[1][8]) - 1e-9 <= r[0][0] <= max(r[0][8], r[1][8]) + 0.05
    import json
    reps = [json.load(open(os.path.join(tmp_path, 'rep%d.json' % k))) for k in range(world)]
    assert reps[0] == reps[1]                # every rank holds the same gathered report
    rep = reps[0]
    assert rep['world_size'] == world and rep['backend'] == 'gloo' and rep['distinct_devices'] == world
    assert [row['rank'] for row in rep['ranks']] == list(range(world))
    for k, row in enumerate(rep['ranks']):
        assert row['env_range'] == [k * E, k * E + E - 1] and row['stacks_per_step'] == 4 * E
        assert abs(row['seconds'] - r[k][8]) < 1e-12 and row['device'] == 'cpu'


def test_rank_report_without_process_group():
    sys.path.insert(0, ROOT)
    import bench
    rep = bench.rank_report({'rank': 0, 'device': 'cpu'}, 1)
    assert rep == {'world_size': 1, 'backend': None, 'ranks': [{'rank': 0, 'device': 'cpu'}], 'distinct_devices': 1}


def test_binding_note_from_committed_stamps():
    """The bench line's roofline.binding comes from the committed stamp profile of the BASELINE
    config (one launch of 64 envs x 4 agents, CHW) and is left out for any other workload."""
    sys.path.insert(0, ROOT)
    import bench
    note = bench.binding_note('lifting_4-small_divider', 256, 'chw')
    assert note is not None and note['resource'].startswith('latency')
    for k in ('sweep_track_us', 'sssp_rounds_us', 'render_track_us', 'join_us', 'distance_phase_us', 'workgroup_total_us'):
        assert 0 < note[k] < 100, k
    assert note['sssp_rounds_us'] < note['sweep_track_us'] < note['join_us'] < note['workgroup_total_us']
    assert bench.binding_note('lifting_4-small_divider', 1024, 'chw') is None
    assert bench.binding_note('pushing_4-large_empty', 256, 'chw') is None


def test_rank_envs_partition():
    sys.path.insert(0, ROOT)
    import bench
    for world in (1, 2, 4, 8):
        ids = [e for r in range(world) for e in bench.rank_envs(r, 128)]
        assert ids == list(range(world * 128))


def _strong_worker(rank, world, port, total, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import bench
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        ids = bench.rank_envs(rank, None, world, total)
        n = int(bench.sum_over_ranks([len(ids)], world)[0])
        # stand-in "states": each env's id in a (2, 3) plane per stack, like the [N, C, 96, 96] output
        out = torch.tensor(ids, dtype=torch.float32).repeat_interleave(2).view(-1, 1, 1).expand(-1, 2, 3).contiguous()
        stats, dst = bench.gather_states(out, 2, world, rank, return_data=True)
        got = None
        if rank == 0:
            got = torch.cat([d[:, 0, 0] for d in dst]).numpy()
        np.save(os.path.join(out_dir, 's%d.npy' % rank),
                np.array([len(ids), ids[0], ids[-1], n, stats['bytes_to_rank0'], stats['reps']]))
        if rank == 0:
            np.save(os.path.join(out_dir, 'gathered.npy'), got)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_strong_split_and_gather(tmp_path):
    """Strong scaling (bench.py --total-envs, BASELINE configs[3] / [4]): an uneven total splits into
    contiguous blocks (4 + 3), the job's stack count sums over ranks, and the optional state gather
    delivers every rank's block to rank 0 (padded to the largest block)."""
    world, total = 2, 7
    mp.spawn(_strong_worker, args=(world, _free_port(), total, str(tmp_path)), nprocs=world, join=True)
    s0, s1 = (np.load(os.path.join(tmp_path, 's%d.npy' % k)) for k in range(world))
    assert list(s0[:4]) == [4, 0, 3, 7] and list(s1[:4]) == [3, 4, 6, 7]
    assert s0[4] == s1[4] == 8 * 2 * 3 * 4 * (world - 1)   # padded block of 4 envs x 2 stacks, f32
    g = np.load(os.path.join(tmp_path, 'gathered.npy'))
    assert list(g) == [0, 0, 1, 1, 2, 2, 3, 3] + [4, 4, 5, 5, 6, 6, 0, 0]


def test_rank_envs_strong_partition():
    sys.path.insert(0, ROOT)
    import bench
    for total in (1024, 2048, 1025, 2047, 9):
        for world in (1, 2, 3, 4, 8):
            blocks = [bench.rank_envs(r, None, world, total) for r in range(world)]
            assert [e for b in blocks for e in b] == list(range(total))
            sizes = [len(b) for b in blocks]
            assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)


def _run_bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, capture_output=True, text=True,
                       env=env, timeout=timeout)
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    return p.returncode, [json.loads(l) for l in lines], p.stderr


@pytest.mark.timeout(300)
def test_bench_main_spawns_its_own_ranks():
    """`bench.py --gpus 2` without a launcher starts its two ranks itself
    (the reference's collector spawns its own workers, train_multiprocess.py:217-228) and the line
    reports both: n_gpus == distributed.world_size == 2, one row per rank, one line in total.  The
    real main() runs end to end with the CPU stand-in launch (--standin) over gloo."""
    rc, lines, err = _run_bench(['--gpus', '2', '--standin', '--steps', '3', '--warmup', '1', '--envs', '2'])
    assert rc == 0, err
    assert len(lines) == 1, lines
    res = lines[0]
    assert res['n_gpus'] == 2 and res['distributed']['world_size'] == 2
    assert res['distributed']['backend'] == 'gloo' and res['distributed']['launcher'] == 'spawn'
    assert [r['rank'] for r in res['distributed']['ranks']] == [0, 1]
    assert [r['env_range'] for r in res['distributed']['ranks']] == [[0, 1], [2, 3]]
    assert res['config']['stacks_per_step'] == 2 * 2 * 4 and res['steps'] == 3
    assert res['data'].startswith('STANDIN') and 'cpu_baseline' not in res


@pytest.mark.timeout(300)
def test_bench_main_single_rank_line():
    """--gpus 1 (and no --gpus) runs in-process: world 1, no process group, launcher 'single'."""
    for extra in (['--gpus', '1'], []):
        rc, lines, err = _run_bench(extra + ['--standin', '--steps', '2', '--warmup', '1', '--envs', '1',
                                             '--no-cpu-baseline'])
        assert rc == 0, err
        assert len(lines) == 1
        res = lines[0]
        assert res['n_gpus'] == 1 and res['distributed']['world_size'] == 1
        assert res['distributed']['backend'] is None and res['distributed']['launcher'] == 'single'


def test_bench_refuses_mismatched_requests():
    """--gpus differing from a launcher's WORLD_SIZE, or more ranks than visible GPUs without
    --shared-gpu, exits non-zero with a message before any timed work."""
    sys.path.insert(0, ROOT)
    import bench
    with pytest.raises(SystemExit, match='WORLD_SIZE=2'):
        bench.resolve_world(3, {'WORLD_SIZE': '2'}, 8)
    with pytest.raises(SystemExit, match='2 ranks requested but 1 GPU'):
        bench.resolve_world(2, {}, 1)
    with pytest.raises(SystemExit, match='>= 1'):
        bench.resolve_world(0, {}, 8)
    assert bench.resolve_world(2, {}, 1, shared_gpu=True) == ('spawn', 2)
    assert bench.resolve_world(8, {}, 8) == ('spawn', 8)
    assert bench.resolve_world(None, {'WORLD_SIZE': '4'}, 8) == ('external', 4)
    assert bench.resolve_world(4, {'WORLD_SIZE': '4'}, 8) == ('external', 4)
    assert bench.resolve_world(None, {}, 1) == ('single', 1)
    assert bench.resolve_world(1, {}, 0, standin=True) == ('single', 1)
    # end to end: this container has no GPU, so two real ranks are refused, non-zero, no line
    rc, lines, err = _run_bench(['--gpus', '2', '--steps', '1', '--warmup', '0'])
    assert rc != 0 and not lines and 'GPU(s) visible' in err
    rc, lines, err = _run_bench(['--gpus', '3', '--standin'], env_extra={'WORLD_SIZE': '2', 'RANK': '0'})
    assert rc != 0 and not lines and 'WORLD_SIZE=2' in err


@pytest.mark.timeout(300)
@pytest.mark.parametrize('config,total', [('lifting_2_throwing_2-large_empty', 10), ('rescue_4-small_empty', 9)])
def test_bench_main_world4_strong_split(config, total):
    """the form the driver's scaling run takes for BASELINE configs[3] / [4]
    (`bench.py --gpus N --config ... --total-envs E`), at world size 4 through the real main()
    (stand-in launch, gloo): n_gpus == world_size == 4, every rank a contiguous block of whole envs,
    the blocks covering 0..E-1 exactly once, and the line strong-scaled over all E envs' stacks."""
    rc, lines, err = _run_bench(['--gpus', '4', '--standin', '--steps', '2', '--warmup', '1', '--config', config,
                                 '--total-envs', str(total)])
    assert rc == 0, err
    assert len(lines) == 1, lines
    res = lines[0]
    d = res['distributed']
    assert res['n_gpus'] == 4 and d['world_size'] == 4 and d['launcher'] == 'spawn'
    assert res['scaling'] == 'strong' and res['config']['total_envs'] == total
    assert res['config']['workload'] == config
    ranges = [row['env_range'] for row in d['ranks']]
    assert [row['rank'] for row in d['ranks']] == [0, 1, 2, 3]
    covered = [e for lo, hi in ranges for e in range(lo, hi + 1)]
    assert covered == list(range(total))  # contiguous, in rank order, each env exactly once
    sizes = [hi - lo + 1 for lo, hi in ranges]
    assert max(sizes) - min(sizes) <= 1
    agents = res['config']['agents_per_env']
    assert res['config']['stacks_per_step'] == total * agents
    assert [row['stacks_per_step'] for row in d['ranks']] == [n * agents for n in sizes]


@pytest.mark.timeout(300)
def test_bench_main_driver_launch_world8():
    """The driver's scaling form at N = 8, verbatim but for the CPU stand-in: `python -m
    torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port P
    bench.py --gpus 8 --steps K --warmup W` (launcher 'external', gloo).  Exactly one JSON line
    (rank 0's), n_gpus == world_size == 8, the default weak split of 64 envs per rank in rank order,
    and value = all ranks' stacks x K / the job time."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')}
    env['OMP_NUM_THREADS'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '8', '--master-addr',
           '127.0.0.1', '--master-port', str(_free_port()), os.path.join(ROOT, 'bench.py'), '--gpus', '8', '--steps',
           '2', '--warmup', '1', '--envs', '2', '--standin']
    p = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout
    res = lines[0]
    d = res['distributed']
    assert res['n_gpus'] == 8 and d['world_size'] == 8 and d['launcher'] == 'external' and d['backend'] == 'gloo'
    assert res['scaling'] == 'weak' and res['steps'] == 2 and res['warmup'] == 1
    assert [row['rank'] for row in d['ranks']] == list(range(8))
    assert [row['env_range'] for row in d['ranks']] == [[2 * r, 2 * r + 1] for r in range(8)]
    assert res['config']['stacks_per_step'] == 8 * 2 * res['config']['agents_per_env']
    slowest = max(row['seconds'] for row in d['ranks'])
    assert res['value'] <= res['config']['stacks_per_step'] * res['steps'] / slowest * (1 + 1e-9)
