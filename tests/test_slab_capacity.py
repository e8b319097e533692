"""Slab buffers that must grow mid-run: with the SPH_SLAB_MINCAP test
hook (read at slab creation) every exchange buffer starts at its minimum and grows to
exactly what a step needs — the particle arrays (Grow), the ghost and migrant send
buffers (the migrant pack is redone after growing), the receive buffers, the NN / SPS
face records and the mDBC face records (sized from the exchange's face counts, so a
record is never dropped).  Each run must be bitwise the run with the default capacities,
and no slab may raise the halo error (ERR_HALO, now fatal and all-reduced)."""
import os

import numpy as np
import pytest

from dualsphysics_multilayer_amd.case import DamBreakCase, WetDambreakNNCase

pytestmark = pytest.mark.gpu


def _with_env(make, mincap):
    old = os.environ.pop("SPH_SLAB_MINCAP", None)
    try:
        if mincap:
            os.environ["SPH_SLAB_MINCAP"] = "1"
        return make()
    finally:
        os.environ.pop("SPH_SLAB_MINCAP", None)
        if old is not None:
            os.environ["SPH_SLAB_MINCAP"] = old


def _case(kind):
    if kind == "verlet":
        c = DamBreakCase(0.025)
        c.vel[c.npb:, 0] = 2.0  # migration across every face
        return c, 3, (4, 0.3, 0.0)
    if kind == "mdbc":
        c = DamBreakCase(0.03, step_algorithm=2, tdensity=1, tboundary=2)
        c.vel[c.npb:, 0] = -1.5
        return c, 3, None
    if kind == "nn":
        return WetDambreakNNCase(0.025, width=0.2, scale=0.5, velgrad=2, tvisco=3, csound=20.0), 2, None
    if kind == "sps":
        c = DamBreakCase(0.03, tvisco=2, visco=1e-6, step_algorithm=2, tdensity=1)
        c.vel[c.npb:, 0] = 1.0
        return c, 3, None
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["verlet", "mdbc", "nn", "sps"])
def test_minimum_slab_capacities_are_bitwise(kind):
    from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition

    case, nslabs, rep = _case(kind)

    def make():
        grp = SphSlabGroup(case, slab_partition(case, nslabs))
        if rep:
            grp.set_repartition(*rep)
        grp.run(16)
        st = grp.stats()
        assert all(s["error_flags"] == 0 for s in st), [s["error_flags"] for s in st]
        return grp.particles()

    ref = _with_env(make, False)
    got = _with_env(make, True)
    for k in ("idp", "pos", "vel", "rhop"):
        assert np.array_equal(got[k], ref[k]), (kind, k)
