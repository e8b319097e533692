"""Symmetry (<parameter Symmetry>, JSph.cpp:714): the plane y = 0 mirrors the particles.
A p1 within 2h of the plane also meets the images of the p2 within 2h of it, visited right
after their originals when those are within the support radius (JSphCpu.cpp:566-613 bound,
671-796 fluid; position y and velocity y mirrored); MapRealPosMin.y = 0 (JSph.cpp:1386); a
particle crossing y = 0 is reflected (JSphCpu.cpp:1247); 2-D, floating bodies and a
viscosity other than the artificial one are refused (JSph.cpp:1174-1179).

Fixtures: the REFERENCE v5.2 CPU solver on the half tank y >= 0 (tests/golden/make_golden.py
SYM_CASES, gencase_ref sym 1: no y = 0 wall, fluid from y = 0).  CPU: the oracle
restatement against them and against the same case without Symmetry; GPU: the HIP core
against them at 10x their own noise floors, on one domain and on slabs, and one interaction
on identical input against the oracle.
"""
import numpy as np
import pytest

from golden_io import boundary, by_idp, cellmode, load, maxdiff, meta, snapshot, steps, tol

from dualsphysics_multilayer_amd.case import DamBreakCase

NAMES = ("verlet_ddt2_sym_dp0.02", "symplectic_ddt1_sym_mdbc_dp0.025")
# with CellMode=half (the images of rows 0 and 1 for a p1 of rows 0 and 1) and with shifting
# (Full: every sum order-free; NoBound: the bound rows in the reference's order, the images
# after them), tests/golden/make_golden.py SYM_EXT_CASES
EXT_NAMES = ("verlet_ddt2_sym_half_dp0.02", "symplectic_ddt2_sym_shift_full_tfs_dp0.025",
             "verlet_ddt2_sym_shift_nobound_dp0.025", "symplectic_ddt2_sym_shift_full_tfs_half_dp0.025")


def case_of(g, **kw):
    dp, step_alg, ddt, _ = meta(g)
    kw.setdefault("symmetry", True)
    kw.setdefault("cellmode", cellmode(g))
    if "ext" in g.files:
        _, _, sh, coef, tfs = g["ext"]
        kw.setdefault("shift_mode", int(sh))
        kw.setdefault("shift_coef", float(coef))
        kw.setdefault("shift_tfs", float(tfs))
    return DamBreakCase(dp, step_algorithm=step_alg, tdensity=ddt, tboundary=boundary(g), **kw)


def gpu_tol(g, k):
    """10x the reference's noise floor on this fixture, at least the tolerances of the
    plain dam break (golden_io.tol; with mDBC those of tests/test_mdbc.py)."""
    if boundary(g) == 2:
        base = (1.4e-8, 2.2e-5, 1e-2) if k <= 1 else ((2e-7, 6e-5, 1e-2) if k <= 20 else (2e-6, 2.1e-4, 2e-2))
    else:
        base = tol(k)
    noise = g["noise_%d" % k] if "noise_%d" % k in g.files else np.zeros(3)
    return tuple(max(b, 10.0 * float(n)) for b, n in zip(base, noise))


def oracle_tol(g, k):
    """2x the noise floor, at least the oracle tolerances of tests/test_oracle_golden.py."""
    base = (1.4e-8, 6e-6, 4e-3) if k <= 1 else ((2e-7, 2e-5, 4e-3) if k <= 20 else (4e-7, 4e-5, 4e-3))
    noise = g["noise_%d" % k] if "noise_%d" % k in g.files else np.zeros(3)
    return tuple(max(b, 2.0 * float(n)) for b, n in zip(base, noise))


def test_case_matches_generator():
    """The half-tank lattice of case.py is gencase_ref's (its PART 0 position hash)."""
    import hashlib

    for n in NAMES + EXT_NAMES:
        g = load(n)
        c = case_of(g)
        assert int(g["symmetry"]) == 1
        pos = c.pos[np.argsort(c.idp, kind="stable")]
        assert hashlib.sha256(np.ascontiguousarray(pos).tobytes()).digest() == bytes(g["s0_sha_pos"])
        assert c.pos[:, 1].min() == 0.0 and c.map_limits()[0][1] == 0.0
        assert c.case_def()["symmetry"] == 1


@pytest.mark.parametrize("name", NAMES)
def test_oracle_symmetry_matches_reference(name):
    oracle = pytest.importorskip("oracle.pyoracle")
    g = load(name)
    o = oracle.OracleSolver(case_of(g), nthreads=4)
    done = 0
    for k in steps(g):
        o.run(k - done)
        done = k
        got, ref = by_idp(o.particles()), snapshot(g, k)
        assert np.array_equal(got["idp"], ref["idp"])
        for q, t in zip(("pos", "vel", "rhop"), oracle_tol(g, k)):
            assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))
        assert abs(o.stats()["time"] - float(ref["time"])) <= 1e-9


def test_symmetry_terms_matter():
    """Without the images the same half tank leaves the reference state far beyond the
    tolerance within 10 steps (so the tests above see the mirror terms)."""
    oracle = pytest.importorskip("oracle.pyoracle")
    g = load(NAMES[0])
    c = case_of(g)
    c.symmetry = False  # the same half-tank lattice, no images (and the default map limits)
    o = oracle.OracleSolver(c, nthreads=4)
    o.run(10)
    got, ref = by_idp(o.particles()), snapshot(g, 10)
    assert np.array_equal(got["idp"], ref["idp"])
    assert maxdiff(got, ref, "vel") > 100 * tol(10)[1]


def test_symmetry_refusals():
    from dualsphysics_multilayer_amd.core import SphError, case_derive

    cd = DamBreakCase(0.05, symmetry=True).case_def()
    bad = dict(cd, tvisco=2, visco=1e-6)
    with pytest.raises(SphError, match="Artificial viscosity"):
        case_derive(bad)
    with pytest.raises(SphError, match="MapRealPosMin"):
        case_derive(dict(cd, map_realposmin=(cd["map_realposmin"][0], -0.01, cd["map_realposmin"][2])))


# ---- HIP path ------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES + EXT_NAMES)
def test_gpu_symmetry_matches_reference(name):
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
@pytest.mark.parametrize("name,nslabs", [(NAMES[0], 3), (NAMES[1], 2), (EXT_NAMES[0], 2), (EXT_NAMES[1], 3)])
def test_gpu_symmetry_slabs_match_reference(name, nslabs):
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
@pytest.mark.parametrize("ddt", [0, 1, 2])
def test_gpu_symmetry_interaction_identical_input(ddt):
    """One interaction with the images on the same developing state, GPU vs oracle, per
    particle within 1e-5 of the array maximum (as test_gpu_parity)."""
    oracle = pytest.importorskip("oracle.pyoracle")
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    case = DamBreakCase(0.0127, tdensity=ddt, celldomfixed=True, symmetry=True)
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


def test_case_xml_symmetry(tmp_path):
    """The run driver's case loader takes <parameter Symmetry> (gencase_ref's XML + bi4):
    MapRealPosMin.y = 0 and the particles of case.py."""
    import os
    import subprocess

    from dualsphysics_multilayer_amd.xmlcase import load_case

    gen = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "gencase_ref")
    if not os.path.exists(gen):
        pytest.skip("oracle/_ref not built")
    subprocess.check_call([gen, "0.04", str(tmp_path), "1", "2", "1.5", "CaseDambreak", "1", "3", "1", "0.1", "0",
                           "-2", "0", "2", "1"], stdout=subprocess.DEVNULL)
    x = load_case(str(tmp_path / "CaseDambreak"))
    cd = x.case_def()
    assert x.symmetry and cd["symmetry"] == 1 and cd["map_realposmin"][1] == 0.0
    ref = DamBreakCase(0.04, symmetry=True)
    assert np.array_equal(np.sort(x.pos, axis=0), np.sort(ref.pos, axis=0))
    assert cd["map_realposmin"] == ref.case_def()["map_realposmin"]


# Symmetry with ShiftMode NoFixed and moving boundaries (the flume's piston and flap, no
# floating box: tests/golden/make_flume_case.py *_sym_nofixed): under NoFixed only a FIXED
# boundary pair freezes the shifting sums, so a moving boundary's image — visited right after
# its original (JSphCpu.cpp:743-750, 793-796) — counts if it comes before the first fixed
# pair: the ordered bound pass stages each row of the first S y rows as [record, image] pairs
# (sph_ext.hip).  Tolerances: the flume's (tests/test_bodies.py).
FLUME_SYM = ("verlet_ddt2_sym_nofixed", "symplectic_ddt1_sym_nofixed")


def _flume_tol(step):
    if step <= 1:
        return 1.4e-8, 2.2e-5, 1e-2
    if step <= 20:
        return 2e-7, 6e-5, 1e-2
    return 2e-6, 2.1e-4, 2e-2


@pytest.mark.parametrize("name", FLUME_SYM)
def test_flume_symmetry_nofixed_case_loaded(name):
    import os

    from dualsphysics_multilayer_amd.xmlcase import XmlCase

    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bi4", "flume_" + name)
    x = XmlCase(os.path.join(d, "CaseFlume"))
    assert x.symmetry and x.shift_mode == 2 and x.case_nmoving == 2 * 176 and x.case_nfloat == 0
    assert x.motion["nobj"] == 2


@pytest.mark.gpu
@pytest.mark.parametrize("name", FLUME_SYM)
def test_gpu_symmetry_nofixed_moving_boundaries_match_reference(name):
    import os

    from dualsphysics_multilayer_amd.core import SphGpuSingle
    from dualsphysics_multilayer_amd.xmlcase import XmlCase

    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bi4", "flume_" + name)
    x = XmlCase(os.path.join(d, "CaseFlume"))
    g = np.load(os.path.join(d, "ref.npz"))
    kept = sorted(int(k[1:].split("_")[0]) for k in g.files if k.startswith("s") and k.endswith("_idp"))
    s = SphGpuSingle(x, device=0)
    done = 0
    for k in kept:
        s.run(k - done)
        done = k
        ref = {q: g["s%d_%s" % (k, q)] for q in ("idp", "pos", "vel", "rhop")}
        got = by_idp(s.particles())
        assert np.array_equal(got["idp"], ref["idp"])
        for q, t in zip(("pos", "vel", "rhop"), _flume_tol(k)):
            assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))
    s.close()
