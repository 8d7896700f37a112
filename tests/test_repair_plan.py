"""CPU: the plan of the byzantine replay (cel_debug_repair_plan, host-only). rsmt2d's
solveCrossword sweeps row i then column i; the device runs that sequence level by level.
Checked on random masks:
  - the solve sequence is the sweep's (an independent Python statement of it);
  - every solve sees, level by level, exactly the cells it sees in the sequence: the known
    cells of its axis when its turn comes = the cells known at the start or filled by a
    solve of a lower level;
  - solves of one level fill disjoint cells and none reads a cell another fills (so one
    launch may run them together)."""
import ctypes

import numpy as np
import pytest


def _plan(mask, k):
    from celestia_eds import _lib
    lib = _lib.load()
    n = 4 * k
    ax, ix, lv = (np.zeros(n, np.int32) for _ in range(3))
    ns, solved = ctypes.c_uint32(0), ctypes.c_int32(0)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    m = np.ascontiguousarray(mask, np.uint8)
    assert lib.cel_debug_repair_plan(P(m), k, P(ax), P(ix), P(lv), ctypes.byref(ns), ctypes.byref(solved)) == _lib.OK
    n = ns.value
    return [(int(a), int(i)) for a, i in zip(ax[:n], ix[:n])], lv[:n].tolist(), bool(solved.value)


def _sweep(mask, k):
    """rsmt2d solveCrossword over the mask alone: (solve sequence, known cells of each
    solve's axis before it, solved)."""
    m = mask.astype(bool).copy()
    w = 2 * k
    seq, seen = [], []
    while True:
        progress = False
        for i in range(w):
            for d in (0, 1):
                line = m[i, :] if d == 0 else m[:, i]
                c = int(line.sum())
                if c == w or c < k:
                    continue
                seq.append((d, i))
                seen.append(frozenset(np.flatnonzero(line).tolist()))
                if d == 0:
                    m[i, :] = True
                else:
                    m[:, i] = True
                progress = True
        if m.all():
            return seq, seen, True
        if not progress:
            return seq, seen, False


@pytest.mark.parametrize("k,p,seed", [(4, 0.5, 1), (8, 0.55, 2), (16, 0.5, 3), (16, 0.4, 4), (32, 0.55, 5),
                                      (64, 0.45, 6), (128, 0.55, 7)])
def test_plan_matches_sweep_and_levels_are_exact(k, p, seed):
    w = 2 * k
    mask = (np.random.default_rng(seed).random((w, w)) < p).astype(np.uint8)
    seq, lv, solved = _plan(mask, k)
    ref, seen, ref_solved = _sweep(mask, k)
    assert seq == ref and solved == ref_solved
    filler_level = np.zeros((w, w), np.int64)  # 0: known at the start
    filled_by = -np.ones((w, w), np.int64)
    m = mask.astype(bool).copy()
    for t, (d, i) in enumerate(seq):
        cells = [(i, j) if d == 0 else (j, i) for j in range(w)]
        for (r, c) in cells:
            if not m[r, c]:
                m[r, c] = True
                filler_level[r, c] = lv[t]
                filled_by[r, c] = t
    for t, (d, i) in enumerate(seq):
        cells = [(i, j) if d == 0 else (j, i) for j in range(w)]
        # known when its level runs: known at the start, or filled by a lower level
        lvl_known = frozenset(j for j, (r, c) in enumerate(cells)
                              if mask[r, c] or (filled_by[r, c] != t and filler_level[r, c] < lv[t]))
        assert lvl_known == seen[t], (t, d, i)
        # nothing it reads or fills is filled by another solve of its level
        for (r, c) in cells:
            o = filled_by[r, c]
            assert o < 0 or o == t or lv[o] != lv[t], (t, o)
