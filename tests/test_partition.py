"""Slab partition (sph_slab_partition, host C++ in the core library; no GPU needed).

The x-columns are split into contiguous slabs of at least 2W columns (W = the ghost width:
1 with full cells, 2 with half cells; two disjoint face column sets per slab) minimising the heaviest slab's weight (fluid + bound_weight x bound particles
per column): checked against an exhaustive dynamic programme on small dam breaks, and
against the prefix-quantile split it replaced (never heavier).
"""
import numpy as np
import pytest

from dualsphysics_multilayer_amd.case import DamBreakCase
from dualsphysics_multilayer_amd.core import case_derive, slab_partition


def column_weights(case, bw=0.3):
    k = case_derive(case.case_def())
    ncx, scell, x0 = int(k["dom_cells"][0]), float(k["scell"]), float(k["dom_posmin"][0])
    dx = case.pos[:, 0] - x0
    cx = np.where(dx >= 0, (dx / scell).astype(np.int64), 0)
    cx = np.minimum(cx, ncx - 1)
    w = np.where(np.arange(case.np) < case.npb, bw, 1.0)
    return np.bincount(cx, weights=w, minlength=ncx), 2 * int(k["scelldiv"])


def best_max_load(w, n, minw):
    """Exhaustive: the smallest possible heaviest slab over contiguous splits."""
    pre = np.concatenate([[0.0], np.cumsum(w)])
    m = len(w)
    inf = float("inf")
    # f[r][c]: best max load splitting columns [0, c) into r slabs
    f = np.full((n + 1, m + 1), inf)
    f[0][0] = 0.0
    for r in range(1, n + 1):
        for c in range(r * minw, m + 1):
            for s in range((r - 1) * minw, c - minw + 1):
                if f[r - 1][s] < inf:
                    f[r][c] = min(f[r][c], max(f[r - 1][s], pre[c] - pre[s]))
    return f[n][m]


def quantile_max_load(w, n, minw):
    pre = np.concatenate([[0.0], np.cumsum(w)])
    m, b, c = len(w), [0], 0
    for r in range(1, n):
        t = pre[m] * r / n
        while c < m and pre[c] < t:
            c += 1
        cut = c - 1 if c > 0 and t - pre[c - 1] < pre[c] - t else c
        cut = min(max(cut, b[-1] + minw), m - (n - r) * minw)
        b.append(cut)
    b.append(m)
    return max(pre[b[r + 1]] - pre[b[r]] for r in range(n))


@pytest.mark.parametrize("dp,cellmode", [(0.02, 1), (0.025, 1), (0.03, 2)])
@pytest.mark.parametrize("nranks", [2, 3, 4])
def test_partition_minimises_the_heaviest_slab(dp, cellmode, nranks):
    case = DamBreakCase(dp, cellmode=cellmode)
    w, minw = column_weights(case)
    b = [int(x) for x in slab_partition(case, nranks)]
    assert b[0] == 0 and b[-1] == len(w)
    assert all(b[r + 1] - b[r] >= minw for r in range(nranks)), b
    pre = np.concatenate([[0.0], np.cumsum(w)])
    got = max(pre[b[r + 1]] - pre[b[r]] for r in range(nranks))
    best = best_max_load(w, nranks, minw)
    assert got <= best * (1 + 1e-9) + 1e-9, (b, got, best)
    assert got <= quantile_max_load(w, nranks, minw) + 1e-9
