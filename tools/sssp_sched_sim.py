"""Host model of the SSSP sweep SCHEDULE in get_state_kernel: the four directional sweeps of one
source run concurrently (timed step by step, not one after the other), rounds end at a barrier,
and two ways to decide what the next round sweeps are compared:

  marks  (the round-3 kernel): a sweep marks the lines it lowered for the opposite direction and
         the lines of its improving lanes for both perpendicular ones; a round ends the rounds when
         it improves nothing -- so the last round only confirms, and lines lowered by a sweep are
         re-swept in the opposite direction even when nothing there can improve;
  check  after every round, one lane-parallel pass over the array tests every edge of every free
         cell, fl(d[u] + w) < d[v] (the fixpoint condition itself); a violated edge u -> v marks
         u's line for the direction(s) whose sweeps relax it.  No violated edge = the fixpoint,
         so there is no confirmation round, and only lines with a real improvement are re-swept.

Both reach the oracle's SPFA fixpoint (asserted).  The output is the critical path of the sweep
waves per source in cycles: per round the slowest wave (its line steps x the step cost of its
cells-per-lane layout), plus a barrier per round, plus the check passes.  The step costs are
HISTORY.md Appendix C's in-kernel measurements (tools/micro/sweep_mb.hip at 8 waves: 148 cycles for
the 2-cells-per-lane step; the 1-cell step runs 9 of its 17 instructions).

    python tools/sssp_sched_sim.py [--config lifting_4-small_divider] [--envs 32]

Test infrastructure only (imports the oracle as the checker).
"""
import argparse
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'spatial-intention-maps_amd'), os.path.join(ROOT, 'oracle')]

S2 = np.float32(np.sqrt(2))
ONE = np.float32(1)
INF = np.float32(np.inf)
DIRS = ('down', 'up', 'right', 'left')
SKIP = None
OPP = {'down': 'up', 'up': 'down', 'right': 'left', 'left': 'right'}


def relax_line(prev, cur, free_cur):
    cand = prev + ONE
    d = prev + S2
    cand[1:] = np.minimum(cand[1:], d[:-1])
    cand[:-1] = np.minimum(cand[:-1], d[1:])
    return np.where(free_cur, np.minimum(cur, cand), cur)


class Sweep:
    """One wave's sweep of one direction over lines [first .. ] with the kernel's stop rule."""

    def __init__(self, dist, free, name, lines, skip=None):
        self.dist, self.free, self.name = dist, free, name
        self.skip = skip            # (min gap in steps, restart cycles): jump over clean gaps
        self.restarts = 0
        H, W = free.shape
        self.vert = name in ('down', 'up')
        n = H if self.vert else W
        fwd = name in ('down', 'right')
        self.order = list(range(n)) if fwd else list(range(n - 1, -1, -1))
        pos = {l: i for i, l in enumerate(self.order)}
        self.dirty = sorted(pos[l] for l in lines)
        self.i = self.dirty[0]
        self.last = self.dirty[-1]
        self.n = n
        self.quiet = 0
        self.steps = 0
        self.improved_lines = []   # (line, improving cell indices)

    def step(self):
        """One line step; False when the sweep is over."""
        if self.i >= self.n - 1:
            return False
        k, k1 = self.order[self.i], self.order[self.i + 1]
        d = self.dist
        if self.vert:
            prev, cur, fr = d[k], d[k1], self.free[k1]
        else:
            prev, cur, fr = d[:, k], d[:, k1], self.free[:, k1]
        new = relax_line(prev.copy(), cur.copy(), fr)
        imp = new < cur
        if self.vert:
            d[k1] = new
        else:
            d[:, k1] = new
        self.steps += 1
        self.i += 1
        if imp.any():
            self.quiet = 0
            self.improved_lines.append((k1, np.nonzero(imp)[0]))
        else:
            self.quiet += 1
            if self.i - 1 >= self.last and self.quiet >= 4:
                return False
            if self.skip and self.quiet >= 4 and (self.steps % 4) == 0:
                # a quiet group: every line up to the next dirty one is clean and unchanged by this
                # sweep, so the sweep may restart there (a new prologue of line prefetches)
                nd = next(p for p in self.dirty if p >= self.i)
                if nd - self.i >= self.skip[0]:
                    self.i = nd
                    self.quiet = 0
                    self.restarts += 1
                    return self.skip[1]
        return True


class RowClose:
    """Judge's round-3 proposal, modelled: a wave that closes whole rows over their straight
    horizontal edges (a DPP min-plus scan left-to-right, then right-to-left, per row: the result of
    the sequential relaxations, which this model applies; diagonals stay with the down / up sweeps).
    One step = one row; its cost is the scan's issue cost (instructions x cycles), the rows being
    independent."""

    def __init__(self, dist, free, name, rows):
        self.dist, self.free, self.name = dist, free, name
        self.rows = sorted(rows)
        self.k = 0
        self.steps = 0
        self.improved_lines = []

    def step(self):
        if self.k >= len(self.rows):
            return False
        r = self.rows[self.k]
        self.k += 1
        row, fr = self.dist[r].copy(), self.free[r]
        W = len(row)
        for j in range(1, W):
            if fr[j] and row[j - 1] + ONE < row[j]:
                row[j] = row[j - 1] + ONE
        for j in range(W - 2, -1, -1):
            if fr[j] and row[j + 1] + ONE < row[j]:
                row[j] = row[j + 1] + ONE
        imp = row < self.dist[r]
        self.dist[r] = row
        self.steps += 1
        if imp.any():
            self.improved_lines.append((r, np.nonzero(imp)[0]))
        return True


def simulate_rowscan(free, src, cost, c_barrier, c_row, waves=2):
    """down / up sweeps (straight + both diagonals) beside `waves` row-closure waves; marks: a
    vertical sweep's lowered rows -> the opposite sweep and the row closure; a closed row that
    improved -> both vertical sweeps.  Ends after a round that improves nothing."""
    H, W = free.shape
    dist = np.full((H, W), INF, np.float32)
    dist[src] = 0
    vm = {'down': {src[0]}, 'up': {src[0]}}
    rows = {src[0]}
    total, rounds, steps = 0.0, 0, {'down': 0, 'up': 0, 'rows': 0}
    cost = dict(cost)
    while True:
        rounds += 1
        objs = {nm: Sweep(dist, free, nm, m) for nm, m in vm.items() if m}
        rl = sorted(rows)
        for q in range(waves):
            part = rl[q::waves]
            if part:
                objs['rows%d' % q] = RowClose(dist, free, 'rows%d' % q, part)
                cost['rows%d' % q] = c_row
        heap = [(cost[nm], nm) for nm in objs]
        heapq.heapify(heap)
        t_end = 0.0
        while heap:
            t, nm = heapq.heappop(heap)
            if objs[nm].step():
                heapq.heappush(heap, (t + cost[nm], nm))
            else:
                t_end = max(t_end, t)
        total += t_end + c_barrier
        vm = {'down': set(), 'up': set()}
        rows = set()
        for nm, o in objs.items():
            key = 'rows' if nm.startswith('rows') else nm
            steps[key] = max(steps[key], 0) + o.steps if key != 'rows' else steps[key] + o.steps
            for line, cells in o.improved_lines:
                if nm.startswith('rows'):
                    vm['down'].add(line)
                    vm['up'].add(line)
                else:
                    vm[OPP[nm]].add(line)
                    rows.add(line)
        if not (vm['down'] or vm['up'] or rows):
            break
        if rounds > 400:
            raise RuntimeError('no convergence')
    return dist, total, rounds, steps


def simulate_async(free, src, cost, c_start, c_poll):
    """No rounds: each direction's wave sweeps again as soon as its own sweep ends (snapshot of its
    dirty lines, c_start cycles of prologue), marking the others at the end of every sweep as the
    round-3 kernel does; an idle wave notices new marks after c_poll cycles.  Done when no sweep
    runs and every mask is empty (the same fixpoint: any schedule of exact relaxations reaches it)."""
    H, W = free.shape
    dist = np.full((H, W), INF, np.float32)
    dist[src] = 0
    masks = {'down': {src[0]}, 'up': {src[0]}, 'right': {src[1]}, 'left': {src[1]}}
    running = {}
    steps = {k: 0 for k in DIRS}
    heap = []
    for nm in DIRS:
        heapq.heappush(heap, (c_start, nm))
    idle = set()
    t_end = 0.0
    sweeps_run = 0
    while heap:
        t, nm = heapq.heappop(heap)
        sw = running.get(nm)
        if sw is None:
            m = masks[nm]
            if not m:
                idle.add(nm)
                continue
            masks[nm] = set()
            running[nm] = sw = Sweep(dist, free, nm, m)
            sweeps_run += 1
        if sw.step():
            heapq.heappush(heap, (t + cost[nm], nm))
            continue
        # the sweep ended: its marks, then the next sweep of this wave
        del running[nm]
        steps[nm] += sw.steps
        vert = nm in ('down', 'up')
        pa, pb = ('right', 'left') if vert else ('down', 'up')
        for line, cells in sw.improved_lines:
            for tgt, val in ((OPP[nm], [line]), (pa, cells.tolist()), (pb, cells.tolist())):
                masks[tgt].update(val)
                if tgt in idle:
                    idle.discard(tgt)
                    heapq.heappush(heap, (t + c_poll, tgt))
        t_end = max(t_end, t)
        heapq.heappush(heap, (t + c_start, nm))
    assert not any(masks.values()) and not running
    return dist, t_end, sweeps_run, steps


def run_round(dist, free, masks, cost, spec=False, skip=None):
    """The round's sweeps, interleaved by time: returns ({dir: Sweep}, round time in cycles).
    spec: a wave whose sweep ended while another's still runs sweeps its direction again over every
    line (speculative; it stops at the next group of 4 steps once the last real sweep ends)."""
    sweeps = {nm: Sweep(dist, free, nm, m, skip) for nm, m in masks.items() if m}
    H, W = free.shape
    heap = [(cost[nm], nm) for nm in sweeps]
    heapq.heapify(heap)
    live = set(sweeps)
    t_end = 0.0
    extra = {}
    spec_dirs = DIRS if spec else ()
    for nm in spec_dirs:   # idle directions start speculating at once
        if nm not in sweeps:
            n = H if nm in ('down', 'up') else W
            extra[nm] = Sweep(dist, free, nm, range(n))
            heapq.heappush(heap, (cost[nm], nm + '*'))
    while heap:
        t, key = heapq.heappop(heap)
        nm = key.rstrip('*')
        if key.endswith('*'):
            if not live:
                continue
            sw = extra[nm]
            if not sw.step():
                n = H if nm in ('down', 'up') else W
                extra[nm] = Sweep(dist, free, nm, range(n))
            heapq.heappush(heap, (t + cost[nm], key))
            continue
        r = sweeps[nm].step()
        if r:
            heapq.heappush(heap, (t + cost[nm] + (0 if r is True else r), nm))
        else:
            t_end = max(t_end, t)
            live.discard(nm)
            if spec and live:
                n = H if nm in ('down', 'up') else W
                extra[nm] = Sweep(dist, free, nm, range(n))
                heapq.heappush(heap, (t + cost[nm], nm + '*'))
    return sweeps, t_end


def violations(dist, free, diag='vert'):
    """Exact fixpoint test of every edge: masks of u-lines per direction that still relax something."""
    H, W = free.shape
    masks = {k: set() for k in DIRS}
    pad = np.full((H + 2, W + 2), INF, np.float32)
    pad[1:-1, 1:-1] = np.where(free, dist, INF)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dy == 0 and dx == 0:
                continue
            w = S2 if dy and dx else ONE
            # edge u -> v with v = u + (dy, dx): u = pad[v - (dy, dx)]
            u = pad[1 - dy:H + 1 - dy, 1 - dx:W + 1 - dx]
            bad = free & (u + w < dist)
            if not bad.any():
                continue
            vr, vc = np.nonzero(bad)
            ur, uc = vr - dy, vc - dx
            if dy == 1:
                masks['down'].update(ur.tolist())
            if dy == -1:
                masks['up'].update(ur.tolist())
            if dy == 0 or diag == 'both':
                if dx == 1:
                    masks['right'].update(uc.tolist())
                if dx == -1:
                    masks['left'].update(uc.tolist())
    return masks


def simulate(free, src, rule, cost, c_barrier, c_check):
    H, W = free.shape
    dist = np.where(free, INF, INF).astype(np.float32)
    dist[src] = 0
    masks = {'down': {src[0]}, 'up': {src[0]}, 'right': {src[1]}, 'left': {src[1]}}
    total = 0.0
    rounds = 0
    per_round = []
    steps = {k: 0 for k in DIRS}
    while True:
        rounds += 1
        sweeps, t = run_round(dist, free, masks, cost, spec=rule.endswith('spec'),
                              skip=SKIP if rule == 'marks_skip' else None)
        total += t + c_barrier
        per_round.append({nm: s.steps for nm, s in sweeps.items()})
        for nm, s in sweeps.items():
            steps[nm] += s.steps
        if rule in ('marks', 'marks_skip', 'perp_final'):
            nxt = {k: set() for k in DIRS}
            any_imp = False
            for nm, s in sweeps.items():
                vert = nm in ('down', 'up')
                pa, pb = ('right', 'left') if vert else ('down', 'up')
                for line, cells in s.improved_lines:
                    any_imp = True
                    if rule in ('marks', 'marks_skip'):
                        nxt[OPP[nm]].add(line)
                    nxt[pa].update(cells.tolist())
                    nxt[pb].update(cells.tolist())
            if rule == 'perp_final' and not any(nxt.values()):
                # no marks left: the exact check decides (perpendicular marks only miss edges back
                # into the line a sweep came from)
                total += c_check
                nxt = violations(dist, free, 'vert')
                if not any(nxt.values()):
                    break
            elif not any_imp:
                break
            masks = nxt
        else:
            total += c_check
            masks = violations(dist, free, 'both' if rule == 'check_both' else 'vert')
            if not any(masks.values()):
                break
        if rounds > 200:
            raise RuntimeError('no convergence')
    return dist, total, rounds, per_round, steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='lifting_4-small_divider')
    ap.add_argument('--envs', type=int, default=32)
    ap.add_argument('--cpl2', type=float, default=148.0, help='cycles per 2-cells-per-lane step')
    ap.add_argument('--cpl1', type=float, default=100.0, help='cycles per 1-cell-per-lane step')
    ap.add_argument('--barrier', type=float, default=300.0, help='cycles per round barrier + masks')
    ap.add_argument('--check', type=float, default=1500.0, help='cycles per check pass + barrier')
    ap.add_argument('--skip-gap', type=int, default=8, help='marks_skip: min clean gap (steps) to jump')
    ap.add_argument('--restart', type=float, default=200.0, help='marks_skip: cycles per restart')
    ap.add_argument('--row-instr', type=float, default=150.0,
                    help='rowscan: instructions per row closure (both scan directions, fast path only)')
    ap.add_argument('--poll', type=float, default=150.0, help='async: cycles for an idle wave to see new marks')
    ap.add_argument('--instr-cycles', type=float, default=6.1, help='issue cycles per instruction')
    args = ap.parse_args()
    global SKIP
    SKIP = (args.skip_gap, args.restart)
    import oracle
    from simaps import synthetic
    res = {r: [] for r in ('marks', 'marks_skip', 'check', 'check_both', 'check_spec', 'perp_final', 'rowscan',
                           'async')}
    detail = {r: [] for r in res}
    for e in range(args.envs):
        sc = synthetic.make_scene(args.config, e)
        for a in range(len(sc['robots'])):
            ao = oracle.AgentOracle(sc, a)
            srcs = [ao.snap(sc['robots'][a]['position'])]
            if sc['receptacle_position'] is not None:
                srcs.insert(0, ao.snap(sc['receptacle_position']))
            rows, cols = np.nonzero(ao.cspace)
            i0, i1, j0, j1 = rows.min(), rows.max() + 1, cols.min(), cols.max() + 1
            free = ao.cspace[i0:i1, j0:j1].astype(bool)
            H, W = free.shape
            cost = {}
            for nm in DIRS:
                span = W if nm in ('down', 'up') else H
                cost[nm] = args.cpl1 if span <= 63 else args.cpl2
            per_agent = {r: 0.0 for r in res}
            for s in srcs:
                ref = oracle.spfa_image(ao.cspace, s)[i0:i1, j0:j1]
                for rule in res:
                    if rule == 'async':
                        d, t, r, st = simulate_async(free, (s[0] - i0, s[1] - j0), cost, args.restart, args.poll)
                        d = np.where(np.isinf(d), np.float32(-1), d)
                        assert np.array_equal(np.where(free, d, 0), np.where(free, ref, 0)), (e, a, rule)
                        per_agent[rule] = max(per_agent[rule], t)
                        detail[rule].append({'rounds': r, 'cycles': t, 'steps': st})
                        continue
                    if rule == 'rowscan':
                        d, t, r, st = simulate_rowscan(free, (s[0] - i0, s[1] - j0), cost, args.barrier,
                                                       args.row_instr * args.instr_cycles)
                        d = np.where(np.isinf(d), np.float32(-1), d)
                        assert np.array_equal(np.where(free, d, 0), np.where(free, ref, 0)), (e, a, rule)
                        per_agent[rule] = max(per_agent[rule], t)
                        detail[rule].append({'rounds': r, 'cycles': t, 'steps': st})
                        continue
                    d, t, r, pr, st = simulate(free, (s[0] - i0, s[1] - j0), rule, cost, args.barrier, args.check)
                    d = np.where(np.isinf(d), np.float32(-1), d)
                    assert np.array_equal(np.where(free, d, 0), np.where(free, ref, 0)), (e, a, rule)
                    per_agent[rule] = max(per_agent[rule], t)   # the two sources run side by side
                    detail[rule].append({'rounds': r, 'cycles': t, 'steps': st})
            for rule in res:
                res[rule].append(per_agent[rule])
    out = {'config': args.config, 'agents': len(res['marks']), 'room': [int(H), int(W)],
           'step_cycles': {'cpl2': args.cpl2, 'cpl1': args.cpl1, 'barrier': args.barrier, 'check': args.check}}
    for rule in res:
        v = np.array(res[rule])
        out[rule] = {'cycles_median': float(np.median(v)), 'cycles_max': float(v.max()),
                     'cycles_p90': float(np.percentile(v, 90)),
                     'rounds_median': float(np.median([d['rounds'] for d in detail[rule]])),
                     'steps_median': {k: float(np.median([d['steps'][k] for d in detail[rule]]))
                                      for k in detail[rule][0]['steps']}}
    for rule in ('marks_skip', 'check', 'check_both', 'check_spec', 'perp_final', 'rowscan', 'async'):
        out[rule + '_vs_marks_median'] = out[rule]['cycles_median'] / out['marks']['cycles_median']
        out[rule + '_vs_marks_max'] = out[rule]['cycles_max'] / out['marks']['cycles_max']
    print(json.dumps(out))


if __name__ == '__main__':
    main()
