"""Loader for the golden fixtures written by tests/golden/make_golden.py."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def steps(g):
    return sorted(int(k[1:].split("_")[0]) for k in g.files if k.endswith("_idp"))


def snapshot(g, step):
    return {k: g["s%d_%s" % (step, k)] for k in ("idp", "pos", "vel", "rhop", "time")}


def meta(g):
    dp, step, ddt, nsteps = g["meta"][:4]
    return float(dp), int(step), int(ddt), int(nsteps)


def boundary(g):
    """1 DBC, 2 mDBC (fixtures written before mDBC carry 4 meta values)."""
    return int(g["meta"][4]) if len(g["meta"]) > 4 else 1


def cellmode(g):
    """1 full, 2 half."""
    return int(g["meta"][5]) if len(g["meta"]) > 5 else 1


def dim(g):
    """3 or 2 (2-D fixtures carry meta[6] = 2)."""
    return int(g["meta"][6]) if len(g["meta"]) > 6 else 3


def kernel(g):
    """1 Cubic spline, 2 Wendland (fixtures without the key)."""
    return int(g["kernel"]) if "kernel" in g.files else 2


def by_idp(p):
    o = np.argsort(p["idp"], kind="stable")
    return {k: (v[o] if isinstance(v, np.ndarray) and v.ndim >= 1 and len(v) == len(o) else v) for k, v in p.items()}


def maxdiff(a, b, key):
    return float(np.abs(a[key].astype(np.float64) - b[key].astype(np.float64)).max())


def tol(step):
    """(pos m, vel m/s, rho kg/m3) GPU-vs-reference tolerance after `step` steps: 10x the
    reference's own rounding-noise floor (step 1 |dx| <= 1e-9 m,
    |dv| <= 2e-5 m/s; step 100 |dx| <= 2e-6 m, |dv| <= 2e-4 m/s, |drho|/rho0 <= 2e-5)."""
    if step <= 1:
        return 1e-9, 2.2e-5, 1e-2
    if step <= 20:
        return 1e-7, 5e-5, 1e-2
    return 2e-6, 2e-4, 2e-2
