"""Host model of the tiled large-window fixpoint (csrc/grid_large.h, gl_tile_kernel): the padded
distance array in global memory, cut into TT x TT tiles; a FIFO of dirty tiles; a tile is processed
by loading it with a one-cell halo, relaxing its edge cells from the (fixed) halo, sweeping its
interior down / up / right / left to its local fixpoint, writing back what fell and marking the
neighbours whose halo changed.  Every value is some path's left-fold float32 length, so the unique
fixpoint -- the reference SPFA's distances (shortest_paths.pyx:69-114) -- is reached; this model
checks that against the oracle bit for bit and counts tile processings / sweep rounds (the GPU
kernel's cost model).

    python tools/tile_sssp_model.py [n] [density] [tile]
"""
import collections
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import oracle  # noqa: E402

S2 = np.float32(np.sqrt(2))
ONE = np.float32(1)
INF = np.float32(np.inf)


def _relax_line(prev, cur):
    """cur[k] = min(cur[k], |prev[k]| + 1, |prev[k -+ 1]| + sqrt2) over one line (float32); the
    line's ends see nothing beyond (the halo was relaxed in beforehand).  Returns True if some
    candidate was below the value read."""
    p = np.abs(prev)
    m = p + ONE
    d = np.full_like(p, INF)
    d[1:] = p[:-1] + S2
    np.minimum(m, d, out=m)
    d[:] = INF
    d[:-1] = p[1:] + S2
    np.minimum(m, d, out=m)
    free = cur != -INF
    better = free & (m < cur)
    if better.any():
        cur[better] = m[better]
        return True
    return False


def local_fixpoint(L, th, tw):
    """Sweep rounds over the interior of L (rows / cols 1..th / 1..tw) until a round changes nothing."""
    rounds = 0
    while True:
        rounds += 1
        ch = False
        I = L[1:th + 1, 1:tw + 1]
        for a in range(1, th):
            ch |= _relax_line(I[a - 1], I[a])
        for a in range(th - 2, -1, -1):
            ch |= _relax_line(I[a + 1], I[a])
        T = I.T  # a view: writes land in L
        for b in range(1, tw):
            ch |= _relax_line(T[b - 1], T[b])
        for b in range(tw - 2, -1, -1):
            ch |= _relax_line(T[b + 1], T[b])
        if not ch:
            return rounds


def pre_relax(L, th, tw):
    """Edge cells from the halo (read-only): straight weight 1, diagonals sqrt2."""
    def relax(i, j, hi, hj, w):
        if L[i, j] == -INF:
            return
        c = np.abs(L[hi, hj]) + w
        if c < L[i, j]:
            L[i, j] = c
    for b in range(1, tw + 1):
        for dj, w in ((-1, S2), (0, ONE), (1, S2)):
            relax(1, b, 0, b + dj, w)
            relax(th, b, th + 1, b + dj, w)
    for a in range(1, th + 1):
        for di, w in ((-1, S2), (0, ONE), (1, S2)):
            relax(a, 1, a + di, 0, w)
            relax(a, tw, a + di, tw + 1, w)


def tiled_image(grid, source, TT=62):
    H, W = grid.shape
    D = np.full((H + 2, W + 2), -INF, np.float32)
    D[1:H + 1, 1:W + 1] = np.where(grid != 0, INF, -INF)
    si, sj = source
    nti, ntj = (H + TT - 1) // TT, (W + TT - 1) // TT
    stats = collections.Counter()
    if grid[si, sj] == 0:
        return None, stats
    # (the source starts at +inf in D and becomes 0 inside its tile's processing, so that it counts as a
    # cell that fell: a source on a tile edge / corner marks the neighbours it is the halo of)
    q = collections.deque([(si // TT, sj // TT)])
    queued = {q[0]}
    while q:
        ti, tj = q.popleft()
        queued.discard((ti, tj))
        r0, c0 = ti * TT, tj * TT
        th, tw = min(TT, H - r0), min(TT, W - c0)
        L = D[r0:r0 + th + 2, c0:c0 + tw + 2].copy()
        old = L[1:th + 1, 1:tw + 1].copy()
        if r0 <= si < r0 + th and c0 <= sj < c0 + tw:
            L[si - r0 + 1, sj - c0 + 1] = 0
        pre_relax(L, th, tw)
        stats['rounds'] += local_fixpoint(L, th, tw)
        stats['tiles'] += 1
        new = L[1:th + 1, 1:tw + 1]
        fell = new < old
        D[r0 + 1:r0 + th + 1, c0 + 1:c0 + tw + 1] = np.minimum(old, new)
        marks = []
        if fell[0].any(): marks.append((ti - 1, tj))
        if fell[-1].any(): marks.append((ti + 1, tj))
        if fell[:, 0].any(): marks.append((ti, tj - 1))
        if fell[:, -1].any(): marks.append((ti, tj + 1))
        if fell[0, 0]: marks.append((ti - 1, tj - 1))
        if fell[0, -1]: marks.append((ti - 1, tj + 1))
        if fell[-1, 0]: marks.append((ti + 1, tj - 1))
        if fell[-1, -1]: marks.append((ti + 1, tj + 1))
        for t in marks:
            if 0 <= t[0] < nti and 0 <= t[1] < ntj and t not in queued:
                queued.add(t)
                q.append(t)
    img = D[1:H + 1, 1:W + 1].copy()
    img[(img == INF) | (img == -INF)] = -1
    img[si, sj] = 0
    return img, stats


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    dens = float(sys.argv[2]) if len(sys.argv) > 2 else 0.25
    TT = int(sys.argv[3]) if len(sys.argv) > 3 else 62
    rs = np.random.RandomState(505)
    grids = {'rand%d' % round(100 * dens): (rs.random_sample((n, n)) > dens).astype(np.uint8)}
    m = np.ones((257, 300), np.uint8)
    m[::8, 1:] = 0
    m[4::16, :-1] = 1
    m[::16, 0] = 1
    m[8::16, -1] = 1
    grids['serpentine'] = m
    for name, g in grids.items():
        free = np.argwhere(g != 0)
        for src in (tuple(free[0]), tuple(free[len(free) // 2])):
            t0 = time.time()
            img, st = tiled_image(g, src, TT)
            ref = oracle.spfa_image(g, src)
            ok = np.array_equal(img.view(np.int32), ref.view(np.int32))
            nt = ((g.shape[0] + TT - 1) // TT) * ((g.shape[1] + TT - 1) // TT)
            print('%s %s src %s: exact %s, %d tiles, %d processings (%.1f per tile), %.2f rounds per processing, %.1f s'
                  % (name, g.shape, src, ok, nt, st['tiles'], st['tiles'] / nt, st['rounds'] / st['tiles'], time.time() - t0))


if __name__ == '__main__':
    main()
