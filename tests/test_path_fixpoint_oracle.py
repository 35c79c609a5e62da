"""CPU: the oracle's restatement of the opt-in fixpoint-parent chain (oracle.fixpoint_chain,
simaps_path_mode 4 / 5) -- every step a tight edge of the f32 fixpoint, the chain's left-fold f32
length from the source equal to D(target) bit for bit (the SPFA's own chain has the same length), and
on the reference's demo sample the same waypoints as the reference within demo.py's atol=2."""
import numpy as np
import pytest

import goldens as G
import oracle as O


def _fold_length(chain):
    acc = np.float32(0)
    for a, b in zip(chain[::-1][:-1], chain[::-1][1:]):
        d = (b[0] - a[0], b[1] - a[1])
        acc = np.float32(acc + O.DIR_LEN[O.DIRS.index(d)])
    return acc


@pytest.mark.parametrize('rule', [1, 2])
def test_fixpoint_chain_is_a_shortest_path(rule):
    rs = np.random.RandomState(7 + rule)
    n = 0
    for dens in (0.0, 0.15, 0.3):
        g = (rs.random_sample((40, 57)) >= dens).astype(np.uint8)
        free = np.argwhere(g)
        for _ in range(12):
            s = tuple(int(x) for x in free[rs.randint(len(free))])
            t = tuple(int(x) for x in free[rs.randint(len(free))])
            d, par = O.spfa(g, s)
            dt = d[t[0] * g.shape[1] + t[1]]
            ch = O.fixpoint_chain(g, s, t, rule)
            assert tuple(ch[0]) == t
            if dt < 0:
                assert len(ch) == 1
                continue
            assert tuple(ch[-1]) == s
            assert _fold_length(ch) == dt
            n += 1
    assert n >= 30


def test_fixpoint_chain_edge_cases():
    g = np.ones((5, 6), np.uint8)
    g[:, 3] = 0  # a wall: the right half is unreachable from the left
    assert O.fixpoint_chain(g, (1, 1), (1, 1), 1) == [[1, 1]]
    assert O.fixpoint_chain(g, (1, 1), (2, 5), 1) == [[2, 5]]      # unreachable
    assert O.fixpoint_chain(g, (1, 1), (2, 3), 2) == [[2, 3]]      # blocked target
    assert np.array(O.grid_shortest_path(g, (1, 1), (2, 5), fixpoint_rule=1)).tolist() == [[2, 5]]


def test_fixpoint_paths_on_the_demo_sample():
    """shortest_paths/demo.py:44-48: the reference's known path within atol=2 under rule 1 (smallest
    D(u) first), as are the reference's three demo-sample paths.  (Rule 2, edge order alone, takes
    another route there: 7 waypoints instead of 6 -- one reason mode 4, not 5, is the one kept.)"""
    rule = 1
    z = G.load('paths.npz')
    demo = G.load('sssp.npz')['demo_cspace']
    path = O.grid_shortest_path(demo, (75, 156), (131, 112), fixpoint_rule=rule)
    correct = np.array([[75, 156], [98, 93], [110, 81], [118, 80], [124, 84], [131, 112]])
    assert np.allclose(np.array(path), correct, atol=2)
    for q in range(3):
        ref = z['demo_%d_path' % q]
        got = np.array(O.grid_shortest_path(demo, tuple(z['demo_%d_src' % q]), tuple(z['demo_%d_tgt' % q]),
                                            fixpoint_rule=rule))
        assert got.shape == ref.shape and np.allclose(got, ref, atol=2), q


def test_edge_order_rule_differs_on_the_demo_sample():
    demo = G.load('sssp.npz')['demo_cspace']
    path = np.array(O.grid_shortest_path(demo, (75, 156), (131, 112), fixpoint_rule=2))
    assert path.shape != (6, 2)
