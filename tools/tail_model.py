"""Model of get_state_kernel's launch tail from a raw per-workgroup stamp table.

A launch lasts from the first workgroup's entry to the last one's end.  This splits that span into
  dispatch   first entry -> this workgroup's entry (stamp 77)
  prologue   entry -> stamp 0 (agents[n] -> envs[ag.env] dependent loads + the first barrier)
  tracks     stamp 0 -> join (stamp 4): max(sweep track end 7, render track end 8) + barrier
  distance   join -> end (stamp 6)
for the median and the slowest workgroups, and asks which per-workgroup quantities predict the
slowest ends: SSSP rounds (stamp 10), sweep line steps per wave (64-71), the binding track, the
entry time.  It also evaluates the two levers of the verdict:
  (a) a prologue with one dependent load instead of two (the env record carried with the agent's),
  (b) no tail beyond the p90 workgroup (the best any per-agent rebalancing could reach),
as predicted launch times, so that an A/B is run only where the model shows >= 3 %.

    python tools/tail_model.py profiles/archive/r5b_stamps.npy [--kernel-us 32.3]
"""
import argparse
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('stamps')
    ap.add_argument('--kernel-us', type=float, default=None, help='rocprofv3 average of the product kernel')
    args = ap.parse_args()
    st = np.load(args.stamps).astype(np.int64)
    us = lambda a: a / 100.0  # noqa: E731  (s_memrealtime: 100 MHz)
    e0 = st[:, 77].min()
    entry = us(st[:, 77] - e0)
    pro = us(st[:, 0] - st[:, 77])
    sweep = us(st[:, 7] - st[:, 0])
    render = us(st[:, 8] - st[:, 0])
    join = us(st[:, 4] - st[:, 0])
    dist = us(st[:, 6] - st[:, 4])
    end = us(st[:, 6] - e0)
    rounds = st[:, 10]
    steps = st[:, 64:72].sum(1)
    span = end.max()
    q = lambda a: [round(float(np.percentile(a, p)), 3) for p in (0, 50, 90, 100)]  # noqa: E731
    slow = np.argsort(-end)[:16]
    binding_sweep = sweep > render
    res = {'workgroups': int(len(st)), 'span_us': round(float(span), 3),
           'percentiles': '0 / 50 / 90 / 100',
           'entry_us': q(entry), 'prologue_us': q(pro), 'sweep_track_us': q(sweep), 'render_track_us': q(render),
           'join_us': q(join), 'distance_us': q(dist), 'end_us': q(end),
           'rounds': {'median': float(np.median(rounds)), 'min': int(rounds.min()), 'max': int(rounds.max())},
           'sweep_binds_frac': round(float(binding_sweep.mean()), 3)}
    # which quantities predict the end of a workgroup (Pearson r over all workgroups)
    feats = {'entry': entry, 'prologue': pro, 'sweep_track': sweep, 'render_track': render, 'rounds': rounds.astype(float),
             'sweep_line_steps': steps.astype(float), 'distance': dist}
    res['corr_with_end'] = {k: round(float(np.corrcoef(v, end)[0, 1]), 3) if v.std() > 0 else None for k, v in feats.items()}
    res['slowest16'] = [{'wg': int(k), 'end': round(float(end[k]), 2), 'entry': round(float(entry[k]), 2),
                         'prologue': round(float(pro[k]), 2), 'sweep': round(float(sweep[k]), 2),
                         'render': round(float(render[k]), 2), 'rounds': int(rounds[k]), 'steps': int(steps[k])}
                        for k in slow]
    # the slowest workgroups against the median one: how much of their excess is each part
    med = np.median(end)
    exc = end[slow] - med
    res['slowest16_excess_us'] = {'end': round(float(np.mean(exc)), 3),
                                  'entry': round(float(np.mean(entry[slow] - np.median(entry))), 3),
                                  'prologue': round(float(np.mean(pro[slow] - np.median(pro))), 3),
                                  'join': round(float(np.mean(join[slow] - np.median(join))), 3),
                                  'distance': round(float(np.mean(dist[slow] - np.median(dist))), 3)}
    # lever (a): one dependent descriptor load fewer in the prologue.  The measured prologue is ~2 load
    # latencies + a barrier; one latency ~ half of (prologue - the barrier's share), taken as
    # (median prologue) / 2.  Whether it shortens a workgroup depends on the binding track: only the
    # part of the saving before the later track's start counts, so both tracks start that much sooner.
    lat = float(np.median(pro)) / 2
    end_a = end - lat
    # lever (b): no workgroup beyond the p90 end
    end_b = np.minimum(end, np.percentile(end, 90))
    res['levers'] = {'descriptor_latency_us': round(lat, 3),
                     'a_one_load_fewer_span_us': round(float(end_a.max()), 3),
                     'a_gain_frac': round(float(1 - end_a.max() / span), 4),
                     'b_tail_cut_to_p90_span_us': round(float(end_b.max()), 3),
                     'b_gain_frac': round(float(1 - end_b.max() / span), 4)}
    if args.kernel_us:
        res['levers']['a_gain_frac_of_kernel'] = round(lat / args.kernel_us, 4)
        res['levers']['b_gain_frac_of_kernel'] = round(float(span - end_b.max()) / args.kernel_us, 4)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
