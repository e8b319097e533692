"""mDBC — modified Dynamic Boundary Conditions.

Reference: JSphCpu::InteractionMdbcCorrectionT2 (JSphCpu.cpp:1020-1187) called before
every interaction except the Symplectic corrector (JSphCpuSingle.cpp:525); normals from
<case>_Normals.nbi4 (JSph::LoadBoundNormals/ConfigBoundNormals, JSph.cpp:1265-1340).

Fixtures (written by the REFERENCE solver and its normals writer JPartNormalData):
  tests/golden/verlet_ddt2_mdbc_dp0.025.npz, symplectic_ddt1_mdbc_dp0.03.npz
      (make_golden.py) — PART snapshots of mDBC dam breaks;
  tests/golden/bi4/mdbc/ (make_mdbc_case.py) — an mDBC case (xml, bi4, _Normals.nbi4)
      and the reference's PART after 20 steps.
The oracle is pinned to these in tests/test_oracle_golden.py (bit-exact after step 1).
CPU tests: the normals file format and the case loader.  GPU tests: the HIP mDBC
kernel against the oracle on the same state (boundary densities, interaction) and
whole runs against the reference PARTs at the GPU tolerance of test_gpu_parity.
"""
import filecmp
import os
import shutil
import subprocess

import numpy as np
import pytest

from golden_io import by_idp, load, maxdiff, meta, snapshot, steps

from dualsphysics_multilayer_amd.case import DamBreakCase
from dualsphysics_multilayer_amd.core import bi4_rewrite, read_normals, read_part, write_normals
from dualsphysics_multilayer_amd.xmlcase import XmlCase

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "bi4", "mdbc")
CASE = os.path.join(FIX, "CaseDambreak")
REF = os.path.join(os.path.dirname(HERE), "oracle", "_ref")
need_ref = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "DualSPHysics5.2CPU_ref")),
                              reason="reference binaries (oracle/_ref) not built here")


# ---- normals file and case loader (CPU) -----------------------------------------------
def test_reference_normals_file_reads_as_generated():
    nor = read_normals(CASE + "_Normals.nbi4")
    assert np.array_equal(nor, DamBreakCase(0.05, tboundary=2).normals_double())


def test_normals_file_rewrite_is_byte_identical(tmp_path):
    dst = str(tmp_path / "n.nbi4")
    bi4_rewrite(CASE + "_Normals.nbi4", dst)
    assert filecmp.cmp(CASE + "_Normals.nbi4", dst, shallow=False)


def test_normals_write_read_round_trip(tmp_path):
    nor = np.random.default_rng(3).normal(size=(57, 3))
    fn = str(tmp_path / "C_Normals.nbi4")
    write_normals(fn, nor, 0.01, 0.0173, "C")
    assert np.array_equal(read_normals(fn), nor)


def test_xml_mdbc_case_is_the_generated_case():
    x, d = XmlCase(CASE), DamBreakCase(0.05, tboundary=2)
    assert x.case_def() == d.case_def()
    assert x.case_def()["tboundary"] == 2 and x.case_def()["slipmode"] == 1
    assert np.array_equal(x.boundnormal, d.boundnormal)
    assert not x.boundnormal[x.npb:].any() and (np.abs(x.boundnormal[: x.npb]).sum(axis=1) > 0).all()


def test_xml_mdbc_restart_refused():
    from dualsphysics_multilayer_amd.xmlcase import CaseError

    with pytest.raises(CaseError, match="extra data"):
        XmlCase(CASE, 20, FIX)


def test_cli_mdbc_options():
    from dualsphysics_multilayer_amd.run import parse_args

    o = parse_args([CASE, "-mdbc", "-mdbc_threshold:0.5", "-mdbc_fast:0"])
    assert o["overrides"]["tboundary"] == 2 and o["overrides"]["mdbc_threshold"] == 0.5
    assert parse_args([CASE, "-dbc"])["overrides"]["tboundary"] == 1


def test_derive_rejects_bad_boundary():
    from dualsphysics_multilayer_amd.core import SphError, case_derive

    cd = DamBreakCase(0.05, tboundary=2).case_def()
    assert case_derive(cd)["tboundary"] == 2
    with pytest.raises(SphError, match="slip mode"):
        case_derive(dict(cd, slipmode=2))
    with pytest.raises(SphError, match="not valid"):
        case_derive(dict(cd, tboundary=3))


@need_ref
def test_reference_reads_our_normals_file(tmp_path):
    """The reference solver run with OUR normals file writes the same PART as with the
    file of its own JPartNormalData."""
    outs = []
    for tag in ("ref", "ours"):
        d = tmp_path / tag
        d.mkdir()
        for f in ("CaseDambreak.xml", "CaseDambreak.bi4"):
            shutil.copy(os.path.join(FIX, f), d / f)
        if tag == "ref":
            shutil.copy(CASE + "_Normals.nbi4", d / "CaseDambreak_Normals.nbi4")
        else:
            write_normals(str(d / "CaseDambreak_Normals.nbi4"), DamBreakCase(0.05, tboundary=2).normals_double(),
                          0.05, DamBreakCase(0.05).h, "CaseDambreak")
        subprocess.check_call([os.path.join(REF, "DualSPHysics5.2CPU_ref"), str(d / "CaseDambreak"), str(d / "out"),
                               "-nsteps:5", "-svsteps:1", "-nortimes:1", "-saveposdouble:1", "-sv:binx", "-svres:0",
                               "-ompthreads:2"], stdout=subprocess.DEVNULL)
        outs.append(by_idp(read_part(str(d / "out" / "Part_0005.bi4"))[1]))
    for k in ("idp", "pos", "vel", "rhop"):
        assert np.array_equal(outs[0][k], outs[1][k]), k


# ---- HIP path (GPU) ----------------------------------------------------------------------
def _gpu(case):
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    return SphGpuSingle(case, device=0)


def _tol(step):
    """10x the reference's own noise floor WITH mDBC: the same solver built with and
    without -ffast-math (the oracle, bit-exact to the reference at step 1) differs from
    the reference by pos 1.4e-9 / vel 1.8e-6 / rho 3.7e-4 after step 1, 1.9e-8 / 6e-6 /
    1.0e-3 after 10-20 steps and 1.8e-7 / 2.1e-5 / 1.8e-3 after 60-100 steps (Verlet DDT2
    and Symplectic DDT1 mDBC goldens) — 2-4x the DBC floor of test_gpu_parity: the
    first-order extrapolation of the boundary density amplifies rounding."""
    if step <= 1:
        return 1.4e-8, 2.2e-5, 1e-2
    if step <= 20:
        return 2e-7, 6e-5, 1e-2
    return 2e-6, 2.1e-4, 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("nsteps", [0, 7])
def test_gpu_mdbc_densities_match_oracle(nsteps):
    """The mDBC kernel on the GPU's state vs the oracle's correction of the same state;
    at t=0 ghost nodes sit on fluid particles (r = 0).  The 4x4 system is solved in
    double on both, but its float inputs (W, gradW, V) differ by a few ulp and the
    first-order extrapolation amplifies them: ~1e-6 relative, the reference's own noise
    floor (1.5e-3 kg/m3)."""
    oracle = pytest.importorskip("oracle.pyoracle")
    case = DamBreakCase(0.03, tboundary=2, celldomfixed=True)
    g, o = _gpu(case), oracle.OracleSolver(case, nthreads=4)
    g.run(nsteps)
    o.run(nsteps)
    assert np.array_equal(g.particles()["idp"], o.particles()["idp"])
    ig, io = g.interaction(), o.interaction()
    pg, po = g.particles(), o.particles()
    nb = case.npb
    rg, ro = pg["rhop"][:nb].astype(np.float64), po["rhop"][:nb].astype(np.float64)
    assert (ro != 1000.0).sum() > 50
    assert np.abs(rg - ro).max() <= (2e-3 if nsteps == 0 else 2e-2), np.abs(rg - ro).max()
    scale = np.abs(io["ace"]).max()
    # the boundary pressures carry those densities (dP = cs0^2 drho ~ 1 Pa); after some
    # steps the two states themselves differ by the mDBC noise floor (see _tol)
    tol = 2e-4 if nsteps == 0 else 1e-3
    assert np.abs(ig["ace"] - io["ace"]).max() <= tol * scale
    # at t=0 ar is DDT round-off (|ar| ~ 0.02 kg/m3/s): an absolute floor of 0.01
    assert np.abs(ig["ar"] - io["ar"]).max() <= tol * np.abs(io["ar"]).max() + 1e-2


@pytest.mark.gpu
def test_gpu_mdbc_ddt1_interaction_matches_oracle():
    """DDT (Molteni) keeps its boundary neighbours under mDBC (JSphCpu.cpp:730)."""
    oracle = pytest.importorskip("oracle.pyoracle")
    case = DamBreakCase(0.03, tboundary=2, tdensity=1, celldomfixed=True)
    g, o = _gpu(case), oracle.OracleSolver(case, nthreads=4)
    g.run(5)
    o.run(5)
    ig, io = g.interaction(), o.interaction()
    # each state after 5 steps carries the mDBC noise floor (see _tol)
    assert np.abs(ig["ar"] - io["ar"]).max() <= 1e-3 * np.abs(io["ar"]).max()
    assert np.abs(ig["ace"] - io["ace"]).max() <= 1e-3 * np.abs(io["ace"]).max()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["verlet_ddt2_mdbc_dp0.025", "symplectic_ddt1_mdbc_dp0.03"])
def test_gpu_mdbc_steps_match_reference_parts(name):
    g_ = load(name)
    dp, step_alg, ddt, _ = meta(g_)
    s = _gpu(DamBreakCase(dp, step_algorithm=step_alg, tdensity=ddt, tboundary=2))
    done = 0
    for k in steps(g_):
        s.run(k - done)
        done = k
        ref = snapshot(g_, k)
        got = by_idp(s.particles())
        assert np.array_equal(got["idp"], ref["idp"]), "excluded-particle set differs"
        tp, tv, tr = _tol(k)
        assert maxdiff(got, ref, "pos") <= tp, (k, maxdiff(got, ref, "pos"))
        assert maxdiff(got, ref, "vel") <= tv, (k, maxdiff(got, ref, "vel"))
        assert maxdiff(got, ref, "rhop") <= tr, (k, maxdiff(got, ref, "rhop"))


@pytest.mark.gpu
def test_gpu_xml_mdbc_case_matches_reference(tmp_path):
    """The XML case (with its _Normals.nbi4) through the run driver for 20 steps vs the
    reference's PART 20."""
    from dualsphysics_multilayer_amd.run import main

    out = str(tmp_path / "out")
    assert main([CASE, out, "-nsteps:20", "-svsteps:1", "-saveposdouble:1", "-sv:binx"]) == 0
    got = by_idp(read_part(os.path.join(out, "Part_0020.bi4"))[1])
    exp = by_idp(read_part(os.path.join(FIX, "Part_0020.bi4"))[1])
    assert np.array_equal(got["idp"], exp["idp"])
    for k, t in zip(("pos", "vel", "rhop"), _tol(20)):
        assert maxdiff(got, exp, k) <= t, (k, maxdiff(got, exp, k))


@pytest.mark.gpu
@pytest.mark.parametrize("nslabs", [2, 4])
def test_gpu_mdbc_on_slabs_matches_reference(nslabs):
    """mDBC on the x-slab decomposition: owned boundary particles only, ghost nodes checked
    to stay inside the slab's grid (their x-normal walls sit at the map ends)."""
    from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition

    g_ = load("verlet_ddt2_mdbc_dp0.025")
    dp, step_alg, ddt, _ = meta(g_)
    case = DamBreakCase(dp, step_algorithm=step_alg, tdensity=ddt, tboundary=2)
    grp = SphSlabGroup(case, slab_partition(case, nslabs))
    done = 0
    for k in steps(g_):
        grp.run(k - done)
        done = k
        ref, got = snapshot(g_, k), grp.particles()
        assert np.array_equal(got["idp"], ref["idp"])
        for q, t in zip(("pos", "vel", "rhop"), _tol(k)):
            assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))
