"""The Cubic spline kernel (TKernel = KERNEL_Cubic): GetKernelCubic_* and its tensile
correction (FunSphKernel.h:38-175), used by the fluid and bound interactions
(JSphCpu.cpp:631-822, the tensile term at :713) and by mDBC (:1020-1187, WabFac).
examples/main/01_DamBreak/CaseDambreak_Def.xml:68 selects it.

Fixtures: the REFERENCE v5.2 CPU solver run with -cubic on the generated dam breaks
(tests/golden/make_golden.py: verlet_ddt2_cubic_dp0.02, symplectic_ddt1_cubic_mdbc_dp0.03,
verlet_ddt2_cubic_2d_dp0.02).  CPU: the oracle restatement against them; GPU: the HIP core
against them at 10x the noise floors of the Wendland fixtures, on one domain and on slabs,
and one interaction on identical input against the oracle.
"""
import numpy as np
import pytest

from golden_io import boundary, by_idp, dim, kernel, load, maxdiff, meta, snapshot, steps, tol

from dualsphysics_multilayer_amd.case import DamBreak2DCase, DamBreakCase

NAMES = ("verlet_ddt2_cubic_dp0.02", "symplectic_ddt1_cubic_mdbc_dp0.03", "verlet_ddt2_cubic_2d_dp0.02")


def case_of(g, **kw):
    dp, step_alg, ddt, _ = meta(g)
    cls = DamBreak2DCase if dim(g) == 2 else DamBreakCase
    return cls(dp, step_algorithm=step_alg, tdensity=ddt, tboundary=boundary(g), kernel=kernel(g), **kw)


def gpu_tol(g, k):
    """10x the reference's own noise floor on THIS fixture (noise_<k>: the fast-math build vs
    the strict build of the same sources, make_golden.py --noise), at least the Wendland
    tolerances: the mDBC ones (tests/test_mdbc.py) with mDBC, else the DBC ones (golden_io.tol).
    (Symplectic + mDBC + Cubic: step-1 floor 4.0e-9 m, vs 3.4e-9 m for the Wendland case.)"""
    if boundary(g) == 2:
        base = (1.4e-8, 2.2e-5, 1e-2) if k <= 1 else ((2e-7, 6e-5, 1e-2) if k <= 20 else (2e-6, 2.1e-4, 2e-2))
    else:
        base = tol(k)
    noise = g["noise_%d" % k] if "noise_%d" % k in g.files else np.zeros(3)
    return tuple(max(b, 10.0 * float(n)) for b, n in zip(base, noise))


def oracle_tol(k):
    """2x the noise floor (tests/test_oracle_golden.py), the mDBC amplification included."""
    return (1.4e-8, 6e-6, 4e-3) if k <= 1 else ((2e-7, 2e-5, 4e-3) if k <= 20 else (4e-7, 4e-5, 4e-3))


def test_fixtures_are_cubic():
    for n in NAMES:
        assert kernel(load(n)) == 1


@pytest.mark.parametrize("name", NAMES)
def test_oracle_cubic_matches_reference(name):
    oracle = pytest.importorskip("oracle.pyoracle")
    g = load(name)
    o = oracle.OracleSolver(case_of(g), nthreads=4)
    done = 0
    for k in steps(g):
        o.run(k - done)
        done = k
        got, ref = by_idp(o.particles()), snapshot(g, k)
        assert np.array_equal(got["idp"], ref["idp"])
        for q, t in zip(("pos", "vel", "rhop"), oracle_tol(k)):
            assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))
        assert abs(o.stats()["time"] - float(ref["time"])) <= 1e-9


def test_cubic_differs_from_wendland():
    """The fixtures are sensitive to the kernel: the Wendland run of the same case leaves
    the Cubic reference state far beyond the tolerance (so the tests above see the kernel)."""
    oracle = pytest.importorskip("oracle.pyoracle")
    g = load(NAMES[0])
    o = oracle.OracleSolver(case_of(g), nthreads=4)
    w = oracle.OracleSolver(DamBreakCase(meta(g)[0], tdensity=meta(g)[2]), nthreads=4)
    o.run(10)
    w.run(10)
    assert maxdiff(by_idp(o.particles()), by_idp(w.particles()), "vel") > 100 * tol(10)[1]


# ---- HIP path ------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_cubic_matches_reference(name):
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    g = load(name)
    s = SphGpuSingle(case_of(g), device=0)
    done = 0
    for k in steps(g):
        s.run(k - done)
        done = k
        got, ref = by_idp(s.particles()), snapshot(g, k)
        assert np.array_equal(got["idp"], ref["idp"])
        for q, t in zip(("pos", "vel", "rhop"), gpu_tol(g, k)):
            assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))
        assert abs(s.stats()["time"] - float(ref["time"])) <= 1e-8 * max(1.0, k)


@pytest.mark.gpu
@pytest.mark.parametrize("name,nslabs", [(NAMES[0], 3), (NAMES[1], 2)])
def test_gpu_cubic_slabs_match_reference(name, nslabs):
    from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition

    g = load(name)
    case = case_of(g)
    grp = SphSlabGroup(case, slab_partition(case, nslabs))
    done = 0
    for k in steps(g):
        grp.run(k - done)
        done = k
        got, ref = grp.particles(), snapshot(g, k)
        assert np.array_equal(got["idp"], ref["idp"])
        for q, t in zip(("pos", "vel", "rhop"), gpu_tol(g, k)):
            assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))


@pytest.mark.gpu
@pytest.mark.parametrize("cellmode", [1, 2])
@pytest.mark.parametrize("ddt", [0, 1, 2, 3])
def test_gpu_cubic_interaction_identical_input(ddt, cellmode):
    """One Cubic interaction (tensile term included) on the same developing state, GPU vs
    oracle, per particle within 1e-5 of the array maximum (as test_gpu_parity)."""
    oracle = pytest.importorskip("oracle.pyoracle")
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    case = DamBreakCase(0.0127, tdensity=ddt, cellmode=cellmode, celldomfixed=True, kernel=1)
    src = SphGpuSingle(case, device=0)
    src.run(40)
    p = by_idp(src.particles())
    assert np.array_equal(p["idp"], np.arange(case.np))
    case.pos[:], case.vel[:], case.rhop[:] = p["pos"], p["vel"], p["rhop"]
    del src
    ig = SphGpuSingle(case, device=0).interaction()
    io = oracle.OracleSolver(case, nthreads=16).interaction()
    assert np.abs(ig["ace"] - io["ace"]).max() <= 1e-5 * np.abs(io["ace"]).max()
    assert np.abs(ig["ar"] - io["ar"]).max() <= 1e-5 * np.abs(io["ar"]).max()
    assert ig["viscdtmax"] == pytest.approx(io["viscdtmax"], rel=1e-5)
    assert ig["acemax"] == pytest.approx(io["acemax"], rel=1e-5)
