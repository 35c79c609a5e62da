"""Per-launch HBM traffic of the ingest kernels from tools/profile_ingest.sh's PMC passes, against
the algorithmic bytes (8 B per camera pixel + 5 B per map pixel, per frame).

    python tools/ingest_traffic.py <tag>    (reads gpurun_out/prof_<tag>_ingest/)

Traffic rule as tools/collect_profiles.py (/opt/skills/guides/MI355X_MICROARCH.md, HBM / rocprofv3):
FETCH_SIZE and WRITE_SIZE (KiB per dispatch) from separate --pmc passes; on gfx950 FETCH_SIZE
reports half the bytes of wide coalesced reads, so it is doubled (an upper estimate for mixed
widths); WRITE_SIZE as reported.  Medians over the profiled launches.
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row['Kernel_Name']
            if 'ingest_' not in name or row['Counter_Name'] != counter:
                continue
            key = 'ingest_points_kernel' if 'points' in name else 'ingest_resolve_kernel'
            out.setdefault(key, []).append(float(row['Counter_Value']))
    return {k: statistics.median(v) for k, v in out.items()}


def main(tag):
    src = os.path.join(ROOT, 'gpurun_out', 'prof_%s_ingest' % tag)
    fetch = per_kernel(os.path.join(src, 'pmc_fetch_counter_collection.csv'), 'FETCH_SIZE')
    write = per_kernel(os.path.join(src, 'pmc_write_counter_collection.csv'), 'WRITE_SIZE')
    bench = json.loads(open(os.path.join(src, 'bench_ktrace.json')).read().strip().splitlines()[-1])
    alg = bench['roofline']['algorithmic_bytes_per_frame'] * bench['frames_per_launch']
    res = {'tag': tag, 'frames_per_launch': bench['frames_per_launch'], 'algorithmic_bytes_per_launch': alg,
           'kernels': {}}
    total = 0.0
    for k in sorted(fetch):
        f2, w = 2 * fetch[k] * 1024, write.get(k, 0.0) * 1024
        res['kernels'][k] = {'fetch_x2_bytes': f2, 'write_bytes': w}
        total += f2 + w
    res['traffic_bytes_per_launch'] = total
    res['traffic_over_algorithmic'] = total / alg
    print(json.dumps(res, indent=1))
    with open(os.path.join(ROOT, 'profiles', '%s_ingest_traffic.json' % tag), 'w') as f:
        json.dump(res, f, indent=1)


if __name__ == '__main__':
    main(sys.argv[1])
