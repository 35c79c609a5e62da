"""Benchmark: agent-state stacks/s of the fused HIP observation path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME] [--envs E]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

A step = one launch rendering every agent of E envs (E x A stacks) from HBM-resident per-agent
maps (inputs uploaded before the timed region).  Multi-GPU: each rank renders its own E envs
(distinct seeds; weak scaling), no data-path collective; barrier + max-over-ranks timing.
Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))

METRIC = 'agent-state-stacks/sec (96\u00d796\u00d7C maps) at 1/2/4/8 MI355X; HBM GB/s vs peak'  # BASELINE.json
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)


def algorithmic_bytes_per_stack(H, W, C):
    """occupancy read H*W (u8) + overhead window 136^2 f32 + state 96^2*C f32."""
    return H * W + 136 * 136 * 4 + 96 * 96 * 4 * C


def cpu_baseline(config, budget_s=15.0):
    """The oracle (numpy + C SPFA restatement of the reference path; 'port') on ONE host core,
    over as many agent stacks of the same workload as fit in ~budget_s seconds (scene generation
    excluded)."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle
    from simaps import synthetic
    oracle.agent_state(synthetic.make_scene(config, 10_000), 0)  # warm: build / load liboracle
    n, e, el = 0, 0, 0.0
    while el < budget_s and e < 100_000:
        s = synthetic.make_scene(config, e)
        for a in range(len(s['robots'])):
            t0 = time.perf_counter()
            oracle.agent_state(s, a)
            el += time.perf_counter() - t0
            n += 1
        e += 1
    return {'value': n / el, 'unit': 'stacks/s', 'cores': 1, 'kind': 'port',
            'sample': '%d agent stacks (%d envs of %s), OccupancyMap.update minus point scatter + '
                      'Mapper.get_state via oracle/ (numpy + C SPFA), 1 thread, %.1f s' % (n, e, config, el)}


def rank_envs(rank, envs_per_rank):
    """Env ids (= scene seeds) of one rank: a contiguous block of whole envs.
    Weak scaling: every rank renders envs_per_rank envs, the job renders world * envs_per_rank."""
    return list(range(rank * envs_per_rank, (rank + 1) * envs_per_rank))


def timed_steps(step, steps, warmup, sync, world, reduce_device='cpu'):
    """The bench contract's timed region: `warmup` untimed steps, then barrier + sync, EXACTLY
    `steps` steps, sync + barrier; returns the wall time, max-reduced over ranks (every rank gets
    the job time).  step(k) runs step k (k < 0 for warmup); sync() waits for the device."""
    import torch
    import torch.distributed as dist
    for k in range(warmup):
        step(-1 - k)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return max_over_ranks([elapsed], world, reduce_device)[0]


def max_over_ranks(values, world, device='cpu'):
    """Element-wise max of per-rank floats (identity for world == 1)."""
    if world == 1:
        return list(values)
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument('--config', default='lifting_4-small_divider')
    ap.add_argument('--envs', type=int, default=64, help='envs per GPU (BASELINE configs[1]: 64)')
    ap.add_argument('--layout', default='chw', choices=['hwc', 'chw'])
    ap.add_argument('--cpu-budget', type=float, default=15.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    from simaps import batch, synthetic
    scenes = [synthetic.make_scene(args.config, e) for e in rank_envs(rank, args.envs)]
    b = batch.StateBatch(scenes, device='cuda', layout=args.layout)
    out = b.alloc_state()
    stream = torch.cuda.current_stream()

    # HIP events on the launch stream bracket the K timed launches (per-launch events would add
    # ~6 us of marker overhead to every step); kernel_ms = their elapsed time / K, i.e. the average
    # launch duration including the launch-to-launch gaps (conservative for the roofline).
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def step(k):
        if k == 0:
            ev0.record(stream)
        b.render(out, stream=stream)
        if k == args.steps - 1:
            ev1.record(stream)

    elapsed = timed_steps(step, args.steps, args.warmup, torch.cuda.synchronize, world, 'cuda')
    kern_ms = max_over_ranks([ev0.elapsed_time(ev1) / args.steps], world, 'cuda')[0]

    stacks_per_step = b.N * world
    value = stacks_per_step * args.steps / elapsed
    B = algorithmic_bytes_per_stack(b.H, b.W, b.C)
    achieved = B * b.N / (kern_ms * 1e-3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    if os.path.exists(tf):
        try:
            t = json.load(open(tf))
            if (t.get('config'), t.get('stacks_per_launch'), t.get('layout')) == (args.config, b.N, args.layout):
                traffic = t.get('hbm_bytes_per_launch')
        except Exception:
            traffic = None

    if rank == 0:
        res = {
            'metric': METRIC,
            'value': value, 'unit': 'stacks/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': elapsed / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic (seeded scenes, SURVEY 8(d))',
            'config': {'workload': args.config, 'envs_per_gpu': args.envs, 'agents_per_env': len(scenes[0]['robots']),
                       'stacks_per_step': stacks_per_step, 'grid': '%dx%d' % (b.H, b.W), 'channels': b.C,
                       'layout': args.layout, 'parallelism': 'env-sharded x%d' % world},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'kernel': 'get_state_kernel', 'kernel_ms': kern_ms,
                         'algorithmic_bytes_per_stack': B},
        }
        if world == 1 and not args.no_cpu_baseline:
            res['cpu_baseline'] = cpu_baseline(args.config, args.cpu_budget)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
