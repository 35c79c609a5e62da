"""Benchmark: agent-state stacks/s of the fused HIP observation path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME] [--envs E | --total-envs T] [--gather R]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

Without a launcher, `--gpus N` (N > 1) starts N rank processes itself (one per GPU, before any GPU
call in the parent); under a launcher, --gpus must equal its WORLD_SIZE.  More ranks than visible
GPUs is refused unless --shared-gpu (a 1-GPU rehearsal over gloo).

A step = one launch rendering every agent of E envs (E x A stacks) from HBM-resident per-agent
maps (inputs uploaded before the timed region).  Multi-GPU: each rank renders its own block of
envs (distinct seeds) -- E per rank (weak scaling, default) or a contiguous share of
--total-envs (strong scaling, BASELINE configs[3] / [4]) -- with no data-path collective; barrier
+ max-over-ranks timing.  --gather R times an optional state gather to rank 0 separately.
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


def cpu_baseline(config, budget_s=6.0, procs=0):
    """the oracle (numpy + C SPFA restatement of the reference path; kind
    "port") on this host's cores -- 1 process and P single-threaded processes -- in a child process
    tree (tools/cpu_baseline.py) that never touches the GPU.  `value` is the P-process aggregate;
    the line also carries the 1-core rate, the CPU model and, from the dev-container calibration
    against the reference itself (profiles/r2_cpu_calibration.json), the reference's estimated rate."""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, 'tools', 'cpu_baseline.py'), '--config', config, '--budget', str(budget_s)]
    if procs:
        cmd += ['--procs', str(procs)]
    out = subprocess.run(cmd, capture_output=True, text=True, check=True, timeout=600)
    return json.loads(out.stdout.strip().splitlines()[-1])


PHASE_PROFILE = os.path.join('profiles', 'phase_binding.json')


def binding_note(config, stacks, layout):
    """How to read roofline.frac: the kernel is latency-bound, not HBM-bound (DESIGN.md section 5,
    'Second roof').  Each of the 256 workgroups renders one stack on its own CU, so a launch lasts as
    long as its workgroups' two concurrent dependency chains -- the SSSP sweep track and the render
    track -- plus the distance phase after their join.  The per-workgroup medians come from the
    committed s_memrealtime stamp profile of the same config / launch size / layout
    (tools/phase_profile.py on the stamp build, summarised into profiles/phase_binding.json), or
    None when there is none."""
    path = os.path.join(ROOT, PHASE_PROFILE)
    try:
        p = json.load(open(path))
    except (OSError, ValueError):
        return None
    if (p.get('config'), p.get('N'), p.get('layout')) != (config, stacks, layout):
        return None
    st, rt = p['sweep_track_us'], p['render_track_us']
    return {'resource': 'latency: per-workgroup dependency chains (SSSP line-to-line sweep recurrence; '
                        'render-track fp64 geometry + barrier-separated phases), one stack per CU',
            'sweep_track_us': st['end'], 'sssp_rounds_us': st['rounds'], 'render_track_us': rt['end'],
            'join_us': p['join_us'], 'distance_phase_us': p['distance_us']['all'],
            'workgroup_total_us': p['total_us_median'], 'sssp_rounds': p['rounds']['median'],
            'source': 'from_profile: %s (%s, stamp build, per-workgroup medians)' % (PHASE_PROFILE, p.get('tag'))}


def rank_envs(rank, envs_per_rank, world=1, total_envs=None):
    """Env ids (= scene seeds) of one rank: a contiguous block of whole envs.
    Weak scaling (total_envs None): every rank renders envs_per_rank envs, the job world *
    envs_per_rank.  Strong scaling: the job renders total_envs envs, split into contiguous blocks
    whose sizes differ by at most one (the first total_envs % world ranks take one more)."""
    if total_envs is None:
        return list(range(rank * envs_per_rank, (rank + 1) * envs_per_rank))
    q, r = divmod(total_envs, world)
    lo = rank * q + min(rank, r)
    return list(range(lo, lo + q + (1 if rank < r else 0)))


START_MARGIN_S = 200e-6  # the agreed start's lead over the latest rank's clock (covers the reduction's return skew)


def timed_steps(step, steps, warmup, sync, world, reduce_device='cpu', own=None):
    """The bench contract's timed region: `warmup` untimed steps, then barrier + sync, EXACTLY
    `steps` steps, sync + barrier; returns the job's wall time (every rank gets it).  step(k) runs
    step k (k < 0 for warmup); sync() waits for the device.  The job's time runs from the EARLIEST
    rank's start (after the opening barrier) to the LATEST rank's end (its sync after its K
    steps): one max-reduction of (-start, end) over the ranks' CLOCK_MONOTONIC stamps
    (time.perf_counter, one clock for every process of the node), so skew between ranks' starts is
    counted.  After the barrier the ranks wait for one agreed start instant, so that skew is the
    clock's, not the barrier's exit.  The closing barrier itself is not: an RCCL barrier costs ~0.1 ms,
    ~15 % of a 20-step region, and is no part of the K steps."""
    import torch
    import torch.distributed as dist
    coll = world > 1 or (dist.is_available() and dist.is_initialized())  # (--init-dist: one rank, real collectives)
    for k in range(warmup):
        step(-1 - k)
    sync()
    if coll:
        dist.barrier()
        # a common start: the ranks leave the barrier up to tens of microseconds apart (host wake-up),
        # so they agree on a start instant on the node's shared CLOCK_MONOTONIC (the latest rank's
        # clock after the barrier + START_MARGIN_S) and each waits for it; a rank that still starts
        # late is counted by the (-start, end) reduction below
        tc = max_over_ranks([time.perf_counter()], world, reduce_device)[0] + START_MARGIN_S
        while time.perf_counter() < tc:
            pass
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    sync()
    t1 = time.perf_counter()
    if coll:
        dist.barrier()
    if own is not None:
        own.append(t1 - t0)  # this rank's own timed region (the rank report)
    neg_start, end = max_over_ranks([-t0, t1], world, reduce_device)
    return end + neg_start


def max_over_ranks(values, world, device='cpu'):
    """Element-wise max of per-rank floats (identity for world == 1 without a process group)."""
    import torch.distributed as dist
    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        return list(values)
    import torch
    t = torch.tensor(values, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu()]


def sum_over_ranks(values, world, device='cpu'):
    """Element-wise sum of per-rank numbers (identity for world == 1 without a process group)."""
    import torch.distributed as dist
    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        return list(values)
    import torch
    t = torch.tensor(values, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.cpu()]


def device_identity(device=None):
    """Which physical GPU this rank renders on: index, name, PCI domain:bus:device (or the device
    UUID when torch does not expose the PCI ids); {'device': 'cpu'} without a GPU (gloo tests)."""
    import torch
    if device is None or getattr(device, 'type', device) == 'cpu' or not torch.cuda.is_available():
        return {'device': 'cpu'}
    idx = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
    p = torch.cuda.get_device_properties(idx)
    out = {'device': 'cuda:%d' % idx, 'name': p.name}
    if all(hasattr(p, a) for a in ('pci_domain_id', 'pci_bus_id', 'pci_device_id')):
        out['pci'] = '%04x:%02x:%02x' % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    elif getattr(p, 'uuid', None) is not None:
        out['pci'] = 'uuid:%s' % p.uuid
    return out


def rank_report(row, world):
    """every rank's own counters (rank, device identity, stacks per step, its timed
    seconds, its kernel ms, ...) all-gathered to every rank, with the process group's own view of
    the job -- its world size and backend -- so that an N-GPU bench line shows by itself that N
    ranks ran on N distinct devices.  Without a process group: the one row, world 1, backend None."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return {'world_size': 1, 'backend': None, 'ranks': [row], 'distinct_devices': 1}
    rows = [None] * dist.get_world_size()
    dist.all_gather_object(rows, row)
    devs = {r.get('pci') or '%s/%s/%s' % (r.get('host'), r.get('device'), r.get('rank')) for r in rows}
    return {'world_size': dist.get_world_size(), 'backend': str(dist.get_backend()), 'ranks': rows,
            'distinct_devices': len(devs)}


def gather_states(out, reps, world, rank, return_data=False):
    """SURVEY.md 8(e)'s optional consumer gather, timed apart from the render: every rank's rendered
    states (padded to the largest block) to rank 0 over RCCL / xGMI, `reps` times; max over ranks.
    (Any device: the gloo tests run it on CPU tensors.)"""
    import torch
    import torch.distributed as dist
    sync = torch.cuda.synchronize if out.is_cuda else (lambda: None)
    n = int(max_over_ranks([out.shape[0]], world, out.device)[0])
    src = torch.zeros((n,) + tuple(out.shape[1:]), dtype=out.dtype, device=out.device)
    src[:out.shape[0]].copy_(out)
    dst = [torch.empty_like(src) for _ in range(world)] if rank == 0 else None
    dist.gather(src, dst, dst=0)  # warm-up (connection setup)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.gather(src, dst, dst=0)
    sync()
    dist.barrier()
    el = max_over_ranks([time.perf_counter() - t0], world, out.device)[0] / reps
    moved = src.numel() * src.element_size() * (world - 1)
    stats = {'ms': el * 1e3, 'bytes_to_rank0': moved, 'GB_per_s': moved / el / 1e9, 'reps': reps,
             'note': 'states of ranks 1..N-1 (padded to the largest block) gathered to rank 0; not in value'}
    return (stats, dst) if return_data else stats


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def resolve_world(gpus, env, device_count, shared_gpu=False, standin=False):
    """How many ranks this invocation runs and who launches them: ('single', 1), ('external', W)
    when a launcher (torch.distributed.run) already set WORLD_SIZE, or ('spawn', N) when
    `bench.py --gpus N` has to start its own N ranks -- the reference's data-parallel collector
    starts its own workers too (train_multiprocess.py:217-228).  Raises SystemExit (non-zero, with
    a message) on a request that cannot be honoured: --gpus different from the launcher's
    WORLD_SIZE, or more ranks than visible GPUs (unless --shared-gpu rehearses them on cuda:0)."""
    if gpus is not None and gpus < 1:
        raise SystemExit('bench.py: --gpus must be >= 1 (got %d)' % gpus)
    if 'WORLD_SIZE' in env:
        world = int(env['WORLD_SIZE'])
        if gpus is not None and gpus != world:
            raise SystemExit('bench.py: --gpus %d but the launcher started WORLD_SIZE=%d ranks' % (gpus, world))
        kind = 'external'
    else:
        world = 1 if gpus is None else gpus
        kind = 'spawn' if world > 1 else 'single'
    if not (shared_gpu or standin) and world > device_count:
        raise SystemExit('bench.py: %d ranks requested but %d GPU(s) visible (--shared-gpu rehearses several '
                         'ranks on cuda:0)' % (world, device_count))
    return kind, world


def spawn_ranks(world, argv, shared_gpu=False):
    """Start `world` child ranks of this script (same arguments), one process per GPU, each with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run would; the parent never
    touches the GPU.  Rank 0's stdout is the bench line.  Returns the first non-zero exit status
    (the other ranks are then terminated) or 0."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK='0' if shared_gpu else str(r), WORLD_SIZE=str(world),
                   LOCAL_WORLD_SIZE=str(world), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                   SIMAPS_BENCH_LAUNCHER='spawn')
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        if live:
            time.sleep(0.05)
    return rc


class StandinBatch:
    """Test-only stand-in for StateBatch (bench.py --standin): the same scenes, slot count and
    output shape, on the CPU, with a render that only fills its output.  It lets the CPU suite run
    bench.main() end to end -- spawn, process group, timed region, rank report, the line -- without
    a GPU; a --standin line says so in `data` and is never a measurement."""

    def __init__(self, scenes, layout):
        from simaps import _lib, batch
        s0 = scenes[0]
        self.N = sum(len(s['robots']) for s in scenes)
        self.H, self.W = s0['H'], s0['W']
        cfg = batch.make_config(s0['flags'], s0['room_width'], s0['room_length'], layout)
        self.C = _lib.lib.simaps_num_channels(cfg, len(s0['robots']))
        self.layout = layout

    def alloc_state(self):
        import torch
        shape = (self.N, self.C, 96, 96) if self.layout == 'chw' else (self.N, 96, 96, self.C)
        return torch.empty(shape, dtype=torch.float32)

    def render(self, out, stream=None):
        out.fill_(1.0)
        return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None,
                    help='ranks (one per GPU); without a launcher bench.py starts them itself (default: 1, or '
                         'the launcher\'s WORLD_SIZE)')
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument('--config', default='lifting_4-small_divider')
    ap.add_argument('--envs', type=int, default=64, help='envs per GPU, weak scaling (BASELINE configs[1]: 64)')
    ap.add_argument('--total-envs', type=int, default=None,
                    help='strong scaling: envs of the whole job, split over the ranks (configs[3]: 1024, [4]: 2048)')
    ap.add_argument('--gather', type=int, default=0, metavar='REPS',
                    help='after the timed region, time REPS gathers of every rank\'s states to rank 0 (reported '
                         'separately, SURVEY.md 8(e))')
    ap.add_argument('--layout', default='chw', choices=['hwc', 'chw'])
    ap.add_argument('--cpu-budget', type=float, default=6.0, help='seconds per CPU-baseline leg and worker')
    ap.add_argument('--cpu-procs', type=int, default=0, help='CPU-baseline processes (default: usable cores, capped)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--init-dist', action='store_true',
                    help='initialise the process group even for one rank (exercises the RCCL init / barrier / '
                         'all_reduce path on a 1-GPU box)')
    ap.add_argument('--shared-gpu', action='store_true',
                    help='rehearsal on a 1-GPU box: every rank renders on cuda:0 and the barriers / reductions go '
                         'over gloo (RCCL refuses two ranks on one device); NOT a scaling measurement')
    ap.add_argument('--standin', action='store_true', help=argparse.SUPPRESS)  # CPU tests only (StandinBatch)
    args = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    # Before any GPU call: decide the ranks, and start them ourselves when no launcher did.
    # (torch.cuda.device_count() does not initialise the GPU on this image.)
    ndev = 0 if args.standin else torch.cuda.device_count()
    kind, world = resolve_world(args.gpus, os.environ, ndev, args.shared_gpu, args.standin)
    if kind == 'spawn':
        return spawn_ranks(world, argv, args.shared_gpu)
    launcher = os.environ.get('SIMAPS_BENCH_LAUNCHER', kind)

    rank = int(os.environ.get('RANK', '0'))
    local = 0 if args.shared_gpu else int(os.environ.get('LOCAL_RANK', '0'))
    cpu = args.standin
    if not cpu:
        torch.cuda.set_device(local)
    red = 'cpu' if (args.shared_gpu or cpu) else 'cuda'  # device of the timing / counter reductions
    dist_on = world > 1 or args.init_dist
    if dist_on:
        if args.shared_gpu or cpu:
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    from simaps import batch, synthetic
    strong = args.total_envs is not None
    if strong and args.total_envs < world:
        raise SystemExit('--total-envs must give every rank at least one env')
    env_ids = rank_envs(rank, args.envs, world, args.total_envs)
    scenes = [synthetic.make_scene(args.config, e) for e in env_ids]
    b = StandinBatch(scenes, args.layout) if cpu else batch.StateBatch(scenes, device='cuda', layout=args.layout)
    out = b.alloc_state()
    stream = None if cpu else torch.cuda.current_stream()

    # HIP events on the launch stream bracket the K timed launches (per-launch events would add
    # ~6 us of marker overhead to every step); kernel_ms = their elapsed time / K, i.e. the average
    # launch duration including the launch-to-launch gaps (conservative for the roofline).
    if not cpu:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def step(k):
        if k == 0 and not cpu:
            ev0.record(stream)
        b.render(out, stream=stream)
        if k == args.steps - 1 and not cpu:
            ev1.record(stream)

    own = []
    sync = (lambda: None) if cpu else torch.cuda.synchronize
    elapsed = timed_steps(step, args.steps, args.warmup, sync, world, red, own)
    own_ms = own[0] * 1e3 / args.steps if cpu else ev0.elapsed_time(ev1) / args.steps
    kern_ms = max_over_ranks([own_ms], world, red)[0]
    import socket
    ident = {'device': 'cpu'} if cpu else device_identity(torch.device('cuda', local))
    ranks = rank_report(dict(ident, rank=rank, local_rank=local,
                             host=socket.gethostname(), env_range=[env_ids[0], env_ids[-1]],
                             stacks_per_step=b.N, steps=args.steps, seconds=own[0], kernel_ms=own_ms), world)
    ranks['launcher'] = launcher

    stacks_per_step = int(sum_over_ranks([b.N], world, red)[0])
    value = stacks_per_step * args.steps / elapsed
    B = algorithmic_bytes_per_stack(b.H, b.W, b.C)
    achieved = B * b.N / (kern_ms * 1e-3) / 1e9
    # HBM traffic comes from rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE cannot be read in-process):
    # the committed profile of the same config / launch size / layout, labelled as such, else null
    traffic, traffic_src = None, None
    tf = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    if os.path.exists(tf):
        try:
            t = json.load(open(tf))
            if (t.get('config'), t.get('stacks_per_launch'), t.get('layout')) == (args.config, b.N, args.layout):
                traffic = t.get('hbm_bytes_per_launch')
                traffic_src = 'from_profile: profiles/pmc_traffic.json (%s, rocprofv3 PMC passes)' % t.get('tag')
        except (OSError, ValueError):
            traffic = None
    binding = binding_note(args.config, b.N, args.layout)
    gather = None
    if args.gather and world > 1:
        gather = gather_states(out.cpu() if args.shared_gpu else out, args.gather, world, rank)

    if rank == 0:
        res = {
            'metric': METRIC,
            'value': value, 'unit': 'stacks/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': elapsed / args.steps * 1e3, 'higher_is_better': True,
            'scaling': 'strong' if strong else 'weak',
            'vs_baseline': None, 'dtype': 'f32',
            'data': 'STANDIN (CPU test of the bench plumbing; not a measurement)' if cpu
                    else 'synthetic (seeded scenes, SURVEY 8(d))',
            'config': {'workload': args.config, 'agents_per_env': len(scenes[0]['robots']),
                       'stacks_per_step': stacks_per_step, 'grid': '%dx%d' % (b.H, b.W), 'channels': b.C,
                       'layout': args.layout,
                       'parallelism': 'env-sharded x%d' % world + (' (shared-gpu rehearsal, gloo)' if args.shared_gpu else '')},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic, 'traffic_source': traffic_src,
                         'kernel': 'get_state_kernel', 'kernel_ms': kern_ms,
                         'algorithmic_bytes_per_stack': B, 'binding': binding},
        }
        res['config'].update({'total_envs': args.total_envs} if strong else {'envs_per_gpu': args.envs})
        res['distributed'] = ranks
        if gather is not None:
            res['gather'] = gather
        if world == 1 and not args.no_cpu_baseline and not cpu:
            res['cpu_baseline'] = cpu_baseline(args.config, args.cpu_budget, args.cpu_procs)
        print(json.dumps(res), flush=True)
    if dist_on:
        dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())
