"""Pins the CPU oracle (oracle/sph_oracle.cpp) to the REFERENCE solver's own output.

Fixtures: PART files written by DualSPHysics v5.2 CPU built from the reference
sources (oracle/Makefile), converted by tests/golden/make_golden.py.

Tolerances: SURVEY.md §4 measured the reference's own rounding-noise floor
(-ffast-math vs strict IEEE build of the same code, 17,295 particles): step 1
|dv| 2.2e-6; step 100 |dx| 1.9e-7 m, |dv| 1.8e-5 m/s, |drho| 1.5e-3 kg/m3.
The oracle must stay inside 2x that floor (it is built with the same flags).
"""
import numpy as np
import pytest

from golden_io import boundary, by_idp, cellmode, load, maxdiff, meta, snapshot, steps

from dualsphysics_multilayer_amd.case import DamBreakCase

oracle = pytest.importorskip("oracle.pyoracle")

CASES = ["verlet_ddt2_dp0.02", "symplectic_ddt1_dp0.025", "verlet_ddtnone_dp0.025", "symplectic_ddt3_dp0.03",
         "verlet_ddt2_mdbc_dp0.025", "symplectic_ddt1_mdbc_dp0.03", "verlet_ddt2_half_dp0.025"]


def tol(step):
    # (pos m, vel m/s, rhop kg/m3): 2x the measured noise floor, interpolated in step count.
    if step <= 1:
        return 1e-8, 6e-6, 2e-3
    if step <= 20:
        return 2e-8, 1e-5, 4e-3
    return 4e-7, 4e-5, 4e-3


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_parts(name):
    g = load(name)
    dp, step_alg, ddt, _ = meta(g)
    case = DamBreakCase(dp, step_algorithm=step_alg, tdensity=ddt, tboundary=boundary(g), cellmode=cellmode(g))
    s = oracle.OracleSolver(case, nthreads=4)
    done = 0
    for k in steps(g):
        s.run(k - done)
        done = k
        ref = snapshot(g, k)
        got = by_idp(s.particles())
        assert np.array_equal(got["idp"], ref["idp"]), "excluded-particle set differs"
        tp, tv, tr = tol(k)
        assert maxdiff(got, ref, "pos") <= tp, (k, maxdiff(got, ref, "pos"))
        assert maxdiff(got, ref, "vel") <= tv, (k, maxdiff(got, ref, "vel"))
        assert maxdiff(got, ref, "rhop") <= tr, (k, maxdiff(got, ref, "rhop"))
        assert abs(s.stats()["time"] - float(ref["time"])) <= 1e-9


def test_oracle_dt_trace_57k():
    g = load("verlet_ddt2_dp0.0127_dt")
    dp, step_alg, ddt, nsteps = meta(g)
    case = DamBreakCase(dp, step_algorithm=step_alg, tdensity=ddt)
    s = oracle.OracleSolver(case, nthreads=8)
    s.run(nsteps)
    dt = s.dt_trace()
    assert len(dt) == nsteps
    assert np.abs(dt / g["dt"] - 1).max() < 2e-6


def test_generator_matches_reference_initial_state():
    import hashlib

    g = load("verlet_ddt2_dp0.02")
    case = DamBreakCase(0.02)
    assert case.np == 17295 and case.npb == 7395
    assert hashlib.sha256(case.pos.tobytes()).digest() == bytes(g["s0_sha_pos"])


def test_oracle_bit_exact_first_step_ddt_none():
    """Step 1 of the DDT-free case: the oracle reproduces the reference's state bit for bit
    (at step 1 all velocities are zero, so the viscosity branch, whose -ffast-math
    rewriting is compiler-specific, does not contribute)."""
    g = load("verlet_ddtnone_dp0.025")
    case = DamBreakCase(0.025, step_algorithm=1, tdensity=0)
    s = oracle.OracleSolver(case, nthreads=3)
    s.run(1)
    ref = snapshot(g, 1)
    got = by_idp(s.particles())
    for k in ("idp", "pos", "vel", "rhop"):
        assert np.array_equal(got[k], ref[k]), k


def test_oracle_mdbc_first_step_bit_exact():
    """mDBC (JSphCpu.cpp:1020-1187): after step 1 of the Verlet mDBC case the oracle's
    state equals the reference's bit for bit — the corrected boundary densities (ghost
    nodes on fluid particles at t=0) feed the boundary pressures of the first
    interaction.  Later steps are covered by the noise-floor test above; the correction
    is active on the walls under the water by step 10."""
    g = load("verlet_ddt2_mdbc_dp0.025")
    case = DamBreakCase(0.025, step_algorithm=1, tdensity=2, tboundary=2)
    s = oracle.OracleSolver(case, nthreads=4)
    s.run(1)
    ref = snapshot(g, 1)
    got = by_idp(s.particles())
    for k in ("idp", "pos", "vel", "rhop"):
        assert np.array_equal(got[k], ref[k]), k
    assert (snapshot(g, 10)["rhop"][: case.npb] != 1000.0).sum() > 100


def test_oracle_mdbc_ghost_on_fluid_particle():
    """At t=0 every ghost node under the water coincides with a fluid particle (r = 0):
    the Wendland gradient factor takes its r -> 0 limit, the extrapolated densities are
    finite and hydrostatic (~rho(z=dp)), as the reference binary computes them."""
    case = DamBreakCase(0.03, tboundary=2)
    s = oracle.OracleSolver(case, nthreads=2)
    s.interaction(1)
    p = by_idp(s.particles())
    rb = p["rhop"][: case.npb]
    assert np.isfinite(rb).all()
    under = (case.pos[: case.npb, 2] == 0) & (case.pos[: case.npb, 0] > 0.05) & (case.pos[: case.npb, 0] < 0.35)
    assert (rb[under] > 1002.0).all() and (rb[under] < 1003.0).all()


def test_oracle_thread_count_independent():
    case = DamBreakCase(0.03)
    runs = []
    for nth in (1, 5):
        s = oracle.OracleSolver(case, nthreads=nth)
        s.run(12)
        runs.append(by_idp(s.particles()))
    for k in ("pos", "vel", "rhop"):
        assert np.array_equal(runs[0][k], runs[1][k]), k
