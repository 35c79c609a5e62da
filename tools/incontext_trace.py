"""Per-phase get_state_kernel durations from a rocprofv3 kernel trace of tools/incontext_probe.py
(the trace's own start / end stamps, independent of where the HIP events sit).

    python tools/incontext_trace.py gpurun_out/prof_<tag>/ktrace_kernel_trace.csv [probe.log]
"""
import csv
import json
import statistics
import sys

PHASES = [('warm', 20), ('back_to_back', 200), ('sync_each', 200), ('gap_100', 200), ('gap_500', 200),
          ('gap_2000', 200), ('update_arrays', 200), ('update_arrays_gap_500', 200)]


def main(path, log=None):
    rows = [r for r in csv.DictReader(open(path)) if 'get_state_kernel' in r['Kernel_Name']]
    n = sum(k for _, k in PHASES)
    rows = rows[len(rows) - n:]
    res, i = {}, 0
    for name, k in PHASES:
        g = rows[i:i + k]
        i += k
        dur = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in g]
        gap = [(int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1e3 for a, b in zip(g, g[1:])]
        res[name] = {'kernel_us_median': round(statistics.median(dur), 2), 'idle_before_us_median': round(statistics.median(gap), 1)}
    out = {'source': path, 'kernel': 'get_state_kernel (lifting_4-small_divider, 256 stacks)', 'phases': res}
    if log:
        for line in open(log):
            if line.startswith('{"probe"'):
                out['hip_event_us_median'] = {k: round(v, 2) for k, v in json.loads(line).items() if k != 'probe'}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:])
