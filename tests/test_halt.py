"""Fatal errors stop a batched run on the device (sph_device.hpp ERR_FATAL).

The reference throws in DtVariable when the computed dt is NaN or infinite
(JSphCpu.cpp:1622) and in RunCellDivide when boundary particles are excluded
(AbortBoundOut), so its run ends at the failing step.  Here a step is a chain of kernels
with no host round trip: once k_dt (or the divide) flags the error, k_dt stops advancing
time and step count and the update / motion / floating kernels leave the state alone, so
sph_solver_run(K) integrates nothing past the failure and sph_solver_sync reports it.
A NaN anywhere in the maxima (VelMax, AceMax, ViscDtMax, ViscEtaDtMax) counts as a NaN dt.
"""
import numpy as np
import pytest

from dualsphysics_multilayer_amd.case import DamBreakCase, WaveFlumeCase

pytestmark = pytest.mark.gpu


def _nan_case(step_algorithm):
    case = DamBreakCase(0.03, step_algorithm=step_algorithm, tdensity=1 if step_algorithm == 2 else 2,
                        celldomfixed=True)
    case.vel = case.vel.copy()
    return case


@pytest.mark.parametrize("step_algorithm", [1, 2])
def test_nan_velocity_stops_at_the_failing_step(step_algorithm):
    from dualsphysics_multilayer_amd.core import SphError, SphGpuSingle

    case = _nan_case(step_algorithm)
    g = SphGpuSingle(case, device=0)
    g.run(5)
    g.sync()
    before = g.particles()
    t5 = g.stats()["time"]
    # a NaN velocity injected through a restart of the same state (the state API)
    pick = int(np.flatnonzero(before["idp"] >= case.npb)[100])
    c2 = case.restart_from(dict(case_nfixed=case.npb, map_posmin=case.map_limits()[0],
                                map_posmax=case.map_limits()[1], timestep=t5), before)
    c2.vel = c2.vel.copy()
    c2.vel[pick] = [np.nan, 0.0, 0.0]
    h = SphGpuSingle(c2, device=0)
    h.set_time(t5, g.stats()["sym_dtpre"])
    p0 = h.particles()
    h.run(10)  # one batch: the first step fails, the other nine must not integrate
    with pytest.raises(SphError, match="Dt is NaN"):
        h.sync()
    st = h.stats()
    assert st["nstep"] == 0, st
    assert st["time"] == t5
    p1 = h.particles()
    o0, o1 = np.argsort(p0["idp"]), np.argsort(p1["idp"])
    assert np.array_equal(p0["idp"][o0], p1["idp"][o1])
    ok = p0["idp"][o0] != p0["idp"][pick]
    # every other particle keeps its state: nothing was integrated after the failure
    assert np.array_equal(p0["pos"][o0][ok], p1["pos"][o1][ok])
    assert np.array_equal(p0["rhop"][o0][ok], p1["rhop"][o1][ok])
    assert np.array_equal(p0["vel"][o0][ok], p1["vel"][o1][ok])


def test_nan_stops_bodies():
    """Moving boundaries and floating bodies do not move after a NaN dt either."""
    from dualsphysics_multilayer_amd.core import SphError, SphGpuSingle

    case = WaveFlumeCase(0.03)
    case.vel = case.vel.copy()
    fl = np.flatnonzero(np.arange(case.np) >= case.case_nbound)
    case.vel[fl[50]] = [0.0, np.nan, 0.0]
    g = SphGpuSingle(case, device=0)
    b0 = g.floatings()
    p0 = g.particles()
    g.run(6)
    with pytest.raises(SphError):
        g.sync()
    assert g.stats()["nstep"] == 0
    b1 = g.floatings()
    for k in ("center", "fvel", "fomega"):
        assert np.array_equal(b0[0][k], b1[0][k]), k
    p1 = g.particles()
    o0, o1 = np.argsort(p0["idp"]), np.argsort(p1["idp"])
    bound = p0["idp"][o0] < case.case_nbound
    assert np.array_equal(p0["pos"][o0][bound], p1["pos"][o1][bound])
