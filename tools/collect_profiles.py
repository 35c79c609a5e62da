"""Copy a round's rocprofv3 summaries from gpurun_out/prof_<tag>/ into profiles/ and derive the
per-launch HBM traffic of get_state_kernel for bench.py's roofline.traffic.

    python tools/collect_profiles.py <tag>

Traffic rule (/opt/skills/guides/MI355X_MICROARCH.md, HBM / rocprofv3 section): FETCH_SIZE and
WRITE_SIZE (KiB per dispatch) come from separate --pmc passes; on gfx950 FETCH_SIZE reports half
the bytes of wide coalesced reads, so it is doubled (our reads are a mix of widths -- the doubled
figure is an upper estimate); WRITE_SIZE counts 16-B-per-lane streaming stores exactly.
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = 'get_state_kernel'


def counter_values(path, name):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if KERNEL in row['Kernel_Name'] and row['Counter_Name'] == name:
                vals.append(float(row['Counter_Value']))
    return vals


def main(tag):
    src = os.path.join(ROOT, 'gpurun_out', 'prof_' + tag)
    dst = os.path.join(ROOT, 'profiles')
    os.makedirs(dst, exist_ok=True)
    for f in ('ktrace_kernel_stats.csv', 'pmc_fetch_counter_collection.csv', 'pmc_write_counter_collection.csv',
              'bench_ktrace.json', 'bench_fetch.json', 'bench_write.json', 'ktrace_agent_info.csv'):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, '%s_%s' % (tag, f)))
    bench = json.loads(open(os.path.join(src, 'bench_ktrace.json')).read().strip().splitlines()[-1])
    avg_ns = None
    with open(os.path.join(src, 'ktrace_kernel_stats.csv')) as f:
        for row in csv.DictReader(f):
            if KERNEL in row['Name']:
                avg_ns = float(row['AverageNs'])
    # per-dispatch durations: the first (cold) launch inflates the stats file's average
    med_ns = None
    trace = os.path.join(src, 'ktrace_kernel_trace.csv')
    if os.path.exists(trace):
        with open(trace) as f:
            durs = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in csv.DictReader(f) if KERNEL in r['Kernel_Name']]
        med_ns = float(statistics.median(durs)) if durs else None
    fetch = counter_values(os.path.join(src, 'pmc_fetch_counter_collection.csv'), 'FETCH_SIZE')
    write = counter_values(os.path.join(src, 'pmc_write_counter_collection.csv'), 'WRITE_SIZE')
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    cfg = bench['config']
    res = {
        'tag': tag, 'kernel': KERNEL, 'config': cfg['workload'], 'stacks_per_launch': cfg['stacks_per_step'],
        'layout': cfg['layout'],
        'fetch_size_kib_median': f_kib, 'write_size_kib_median': w_kib,
        'hbm_bytes_per_launch': int(round((2 * f_kib + w_kib) * 1024)),
        'algorithmic_bytes_per_launch': bench['roofline']['algorithmic_bytes_per_stack'] * cfg['stacks_per_step'],
        'rocprof_avg_kernel_ns': avg_ns, 'rocprof_median_kernel_ns': med_ns,
        'bench_event_kernel_ms': bench['roofline']['kernel_ms'],
        'rule': 'traffic = 2 * FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md)',
    }
    json.dump(res, open(os.path.join(dst, 'pmc_traffic.json'), 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(sys.argv[1])
