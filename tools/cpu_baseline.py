"""CPU baseline of the observation path: the oracle (numpy + the C SPFA
restatement of envs.py:2445-2466 + 2068-2185 and shortest_paths.pyx:69-114; kind "port") timed on
this host's cores, in 1 process and in P processes (one single-threaded worker per core).

    python tools/cpu_baseline.py --config lifting_4-small_divider --budget 6 --procs P

Prints one JSON object.  Runs in its own process tree (bench.py starts it as a child before it
touches the GPU's results), so the workers can fork freely.  Scene generation is excluded from the
timed region; each worker renders whole envs (all agents) of distinct seeds until its budget ends.
The port / reference speed ratio measured in the dev container (tools/cpu_calibration.py ->
profiles/r2_cpu_calibration.json) converts the port's rate into an estimate of the reference's.
"""
import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORIG_OMP = os.environ.get('OMP_NUM_THREADS', '')  # the job's thread budget (16 on a one-GPU box)
for _v in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS'):
    os.environ[_v] = '1'  # one thread per worker (set before numpy loads)
sys.path.insert(0, os.path.join(ROOT, 'spatial-intention-maps_amd'))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))

CALIBRATION = os.path.join(ROOT, 'profiles', 'r2_cpu_calibration.json')


def cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or 'unknown'


def worker(args):
    config, wid, stride, budget = args
    import oracle
    from simaps import synthetic
    oracle.agent_state(synthetic.make_scene(config, 1_000_000 + wid), 0)  # warm: load liboracle, caches
    n, e, el = 0, wid, 0.0
    while el < budget:
        s = synthetic.make_scene(config, e)
        for a in range(len(s['robots'])):
            t0 = time.perf_counter()
            oracle.agent_state(s, a)
            el += time.perf_counter() - t0
            n += 1
        e += stride
    return n, el


def default_procs():
    """Cores this process may use, capped by the job's thread budget (OMP_NUM_THREADS as the
    environment set it before this module forced 1, e.g. 16 on a one-GPU box)."""
    cap = int(os.environ.get('SIMAPS_CPU_PROCS', '0') or 0) or (int(ORIG_OMP) if ORIG_OMP.isdigit() else 0)
    n = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    return max(1, min(n, cap) if cap else n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='lifting_4-small_divider')
    ap.add_argument('--budget', type=float, default=6.0, help='seconds of timed work per worker and leg')
    ap.add_argument('--procs', type=int, default=0, help='parallel workers (default: usable cores, capped)')
    args = ap.parse_args()
    P = args.procs or default_procs()
    n1, t1 = worker((args.config, 0, 1, args.budget))
    one = n1 / t1
    t0 = time.perf_counter()
    with mp.get_context('fork').Pool(P) as pool:
        res = pool.map(worker, [(args.config, 10_000 + w, P, args.budget) for w in range(P)])
    wall = time.perf_counter() - t0
    nP = sum(r[0] for r in res)
    # aggregate = sum of the workers' own rates (each timed over its stacks only)
    agg = sum(r[0] / r[1] for r in res)
    out = {'value': agg, 'unit': 'stacks/s', 'cores': P, 'kind': 'port', 'cpu': cpu_model(),
           'one_core': one,
           'sample': '%s: 1 process %d stacks in %.1f s; %d processes x ~%.0f s, %d stacks (wall %.1f s incl. scene '
                     'generation); OccupancyMap.update minus point scatter + Mapper.get_state via oracle/ '
                     '(numpy + C SPFA), 1 thread per process' % (args.config, n1, t1, P, args.budget, nP, wall)}
    if os.path.exists(CALIBRATION):
        cal = json.load(open(CALIBRATION))
        r = cal.get(args.config, {}).get('port_over_reference')
        if r:
            out['calibration'] = {'port_over_reference': r, 'measured': cal.get('host', ''),
                                  'source': os.path.relpath(CALIBRATION, ROOT)}
            out['reference_estimate'] = {'one_core': one / r, 'all_cores': agg / r}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
