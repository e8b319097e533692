"""NN multiphase (the v5.0 NNewtonian solver; SURVEY.md §8(f) row 4, BASELINE cfg5).

Parity is pinned directly to the REFERENCE v5.0 NN solver built from its sources
(oracle/Makefile -> oracle/_ref/DualSPHysics5.0NN_CPU_ref): tests/golden/make_nn_golden.py
runs it on the 3-D extruded wet dam break that oracle/tools/gennn_ref writes and stores its
PARTs, plus the reference's own rounding-noise floor (the same sources built without
-ffast-math, noise_<step>).  The GPU core (through the C-ABI) is held to 10x that floor,
with a floor of a few float ulps where the two reference builds agree bit for bit.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from golden_io import GOLDEN, by_idp, maxdiff, snapshot, steps

from dualsphysics_multilayer_amd.case import WetDambreakNNCase

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
NN_GOLDENS = ("sym_lam_dp0.02", "sym_consteq_cs_dp0.025", "ver_art_ddt1_cs_dp0.025")
# VelocityGradientType 2 (SPH velocity gradients: k_nn_tiled<4|5> then k_nn_visc)
NN_SPH_GOLDENS = ("sph_sym_lam_dp0.02", "sph_sym_consteq_cs_dp0.025", "sph_ver_lam_ddt1_nobound_dp0.025",
                  "sph_ver_art_cs_dp0.025")
# CellMode=half (-cellmode:half, JCellSearch_inline.h:38-44: cells of h, 5x5 rows)
NN_HALF_GOLDENS = ("sym_lam_half_dp0.02", "sph_sym_consteq_cs_half_dp0.025", "ver_art_ddt1_cs_half_dp0.025")
# ulp-level floors (pos m, vel m/s, rho kg/m3): 10x noise of exactly 0 is no tolerance
FLOOR = (2e-10, 2e-8, 2.5e-3)


def load_nn(name):
    return np.load(os.path.join(GOLDEN, "nn_%s.npz" % name))


def case_of(g):
    dp, width, scale, tfs, vg, tv, ddt, sh, cs, step, _ = g["meta"]
    return WetDambreakNNCase(float(dp), width=float(width), scale=float(scale), shift_tfs=float(tfs),
                             tvisco=int(tv), tdensity=int(ddt), shift_mode=int(sh), csound=float(cs),
                             step_algorithm=int(step), velgrad=int(vg),
                             cellmode=int(g["cellmode"]) if "cellmode" in g.files else 1)


# CellMode=half: 25 rows per pass drained in 12 mirrored pairs + the own row, against the
# reference's z-major order of 25 rows, moves the step-1 positions by up to ~3e-10 m (the
# sums' rounding; fast-math vs strict builds of the reference keep the order, so their noise
# floor does not show this)
FLOOR_HALF = (5e-10, 2e-8, 2.5e-3)


def nn_tol(g, k):
    n = g["noise_%d" % k]
    fl = FLOOR_HALF if "cellmode" in g.files and int(g["cellmode"]) == 2 else FLOOR
    return tuple(max(10.0 * float(n[i]), fl[i]) for i in range(3))


# ---- CPU ----------------------------------------------------------------------------------
@pytest.mark.parametrize("name", NN_GOLDENS + NN_SPH_GOLDENS + NN_HALF_GOLDENS)
def test_goldens_present_with_noise_floor(name):
    g = load_nn(name)
    ks = steps(g)
    assert ks and all(("noise_%d" % k) in g.files for k in ks)
    for k in ks:
        assert np.all(np.isfinite(g["noise_%d" % k]))


def test_case_generator_matches_gennn_ref(tmp_path):
    """The product-side generator equals the reference-side one (particles, order, codes of the
    fluid blocks, constants as the case XML stores them)."""
    exe = os.path.join(REF, "gennn_ref")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built")
    from dualsphysics_multilayer_amd.core import read_part

    out = subprocess.check_output([exe, "0.025", str(tmp_path), "0.2", "0.5", "5", "CaseNN", "2.75", "1", "2", "3",
                                   "3", "20"], text=True)
    fields = dict(kv.split("=") for kv in out.split())
    c = WetDambreakNNCase(0.025, width=0.2, scale=0.5, csound=20.0)
    assert int(fields["np"]) == c.np and int(fields["nb"]) == c.npb
    assert [int(fields["nph%d" % k]) for k in range(3)] == c.nph
    hdr, parts = read_part(str(tmp_path / "CaseNN.bi4"))
    assert np.array_equal(parts["idp"], c.idp)
    assert np.array_equal(parts["pos"], c.pos)
    xml = open(tmp_path / "CaseNN.xml").read()
    import re

    xv = {k: float(re.search(r'<%s value="([^"]+)"' % k, xml).group(1)) for k in ("h", "b", "massfluid")}
    assert (xv["h"], xv["b"], xv["massfluid"]) == (c.h, c.cteb, c.mass)
    assert '<csound value="22"/>' in xml  # phase 1: csound*(1+0.1)
    assert c.phases[1]["cs0"] == 22.0


def test_derived_constants_match_reference_log():
    """Values printed by the v5.0 reference's Run.out for the sym_lam_dp0.02 case:
    Cs0=20, DtIni=0.00159217, DtMin=7.96085e-10 (CoefDtMin x 1e-5, ConfigConstantsMP)."""
    from dualsphysics_multilayer_amd.core import case_derive

    k = case_derive(WetDambreakNNCase(0.02, width=0.2, scale=0.5).case_def())
    assert k["cs0"] == pytest.approx(20.0, rel=1e-7)
    assert k["dtini"] == pytest.approx(0.00159217, rel=1e-5)
    assert k["dtmin"] == pytest.approx(7.96085e-10, rel=1e-5)
    assert k["rheology"] == 2 and k["nphases"] == 3
    # phase masses rho dp^3 and CteB = Cs0^2 rho/gamma (ConfigConstantsMP without <csound>)
    assert k["phase_mass"][:3] == pytest.approx([0.016, 0.012, 0.008], rel=1e-6)
    assert k["phase_cteb"][:3] == pytest.approx([400 * 2000 / 7, 400 * 1500 / 7, 400 * 1000 / 7], rel=1e-6)


def test_invalid_nn_configurations_rejected():
    from dualsphysics_multilayer_amd.core import case_derive

    base = WetDambreakNNCase(0.05, width=0.2, scale=0.5)
    d = base.case_def()
    d["tboundary"] = 2
    with pytest.raises(RuntimeError, match="mDBC"):
        case_derive(d)
    d = base.case_def()
    d["nphases"] = 0
    with pytest.raises(RuntimeError, match="phases"):
        case_derive(d)
    d = base.case_def()
    d["velgrad"] = 3
    with pytest.raises(RuntimeError, match="gradient"):
        case_derive(d)


# ---- GPU ----------------------------------------------------------------------------------
def gpu(case):
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    return SphGpuSingle(case, device=0)


def check(got, ref, tol, k):
    assert np.array_equal(got["idp"], ref["idp"]), "excluded-particle set differs"
    for q, t in zip(("pos", "vel", "rhop"), tol):
        assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q), t)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NN_GOLDENS + NN_SPH_GOLDENS + NN_HALF_GOLDENS)
def test_gpu_nn_steps_match_reference_parts(name):
    g = load_nn(name)
    s = gpu(case_of(g))
    done = 0
    for k in steps(g):
        s.run(k - done)
        done = k
        ref = snapshot(g, k)
        check(by_idp(s.particles()), ref, nn_tol(g, k), k)
        assert abs(s.stats()["time"] - float(ref["time"])) <= 1e-9 * max(1.0, k)


@pytest.mark.gpu
def test_gpu_nn_dt_trace_matches_reference():
    g = load_nn("sym_lam_dp0.02")
    s = gpu(case_of(g))
    n = len(g["dt"])
    s.run(n)
    dt = s.dt_trace()
    assert len(dt) == n
    assert np.abs(dt / g["dt"] - 1).max() < 1e-5
    assert s.stats()["viscetadtmax"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("nslabs,name", [(2, "sym_lam_dp0.02"), (2, "sph_sym_lam_dp0.02"), (3, "sph_sym_consteq_cs_dp0.025"),
                                         (2, "sym_lam_half_dp0.02"), (3, "sph_sym_consteq_cs_half_dp0.025")])
def test_gpu_nn_slabs_match_reference_parts(nslabs, name):
    """Slabs; with SPH gradients the first pass's eta / tau of the face columns go to the
    neighbours' ghosts before the second pass (NNFaceExchange)."""
    from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition

    g = load_nn(name)
    case = case_of(g)
    grp = SphSlabGroup(case, slab_partition(case, nslabs))
    done = 0
    for k in steps(g):
        grp.run(k - done)
        done = k
        check(grp.particles(), snapshot(g, k), nn_tol(g, k), k)
        times = [st["time"] for st in grp.stats()]
        assert max(times) == min(times)


@pytest.mark.gpu
def test_gpu_nn_deterministic():
    case = WetDambreakNNCase(0.025, width=0.2, scale=0.5)
    a, b = gpu(case), gpu(case)
    a.run(20)
    b.run(20)
    pa, pb = a.particles(), b.particles()
    for q in ("idp", "pos", "vel", "rhop"):
        assert np.array_equal(pa[q], pb[q]), q


@pytest.mark.parametrize("velgrad", [1, 2])
def test_xml_loader_reads_the_nn_case(tmp_path, velgrad):
    """xmlcase (the run driver's JSph::LoadCaseConfig) reads gennn_ref's case for the v5.0
    solver — RheologyTreatment, VelocityGradientType, ViscoTreatment, shifting, RelaxationDt
    and <special><nnphases> — into the same SphCaseDef and particle codes as the generator."""
    exe = os.path.join(REF, "gennn_ref")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built")
    from dualsphysics_multilayer_amd.xmlcase import XmlCase

    subprocess.check_call([exe, "0.025", str(tmp_path), "0.2", "0.5", "5", "CaseNN", "2.75", str(velgrad), "3", "1", "1",
                           "20"], stdout=subprocess.DEVNULL)
    x = XmlCase(str(tmp_path / "CaseNN"))
    c = WetDambreakNNCase(0.025, width=0.2, scale=0.5, csound=20.0, tvisco=3, tdensity=1, shift_mode=1,
                          velgrad=velgrad)
    assert x.case_def() == c.case_def()
    assert np.array_equal(x.code, c.code) and np.array_equal(x.idp, c.idp)
    assert np.array_equal(x.pos, c.pos)


# ---- NN multiphase with a floating body (JSphCpu_NN_FDA.cpp:89-93, 159-164, 203-215) ------
# gennn_ref float 1 (a box of rhopbody 800 on the phase-0 layer); make_nn_golden.py ft_* runs
# the REFERENCE v5.0 NN solver on it.  The case comes back through the run driver's loader
# (xmlcase), which configures the body as JSph::LoadCaseConfig does.
NN_FT_GOLDENS = ("ft_sym_lam_ddt3_dp0.025", "ft_ver_art_ddt1_nobound_cs_dp0.025", "ft_sph_sym_consteq_cs_dp0.025",
                 # CellMode=half (the npz carries cellmode = 2)
                 "ft_sym_lam_ddt3_half_dp0.025", "ft_ver_art_ddt1_nobound_cs_half_dp0.025",
                 # external forces on the body and a ViscoTime table (the npz carries xmledit)
                 "ft_sym_lam_ddt3_extforce_viscotime_dp0.025")


def ft_case(g, tmp_path):
    from dualsphysics_multilayer_amd.xmlcase import XmlCase

    exe = os.path.join(REF, "gennn_ref")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built")
    dp, width, scale, tfs, vg, tv, ddt, sh, cs, step, _ = g["meta"]
    subprocess.check_call([exe, repr(float(dp)), str(tmp_path), repr(float(width)), repr(float(scale)), "5", "CaseNN",
                           repr(float(tfs)), str(int(vg)), str(int(tv)), str(int(ddt)), str(int(sh)), repr(float(cs)),
                           str(int(step)), "1"], stdout=subprocess.DEVNULL)
    if "xmledit" in g.files:  # the generator's XML edit and data files (make_nn_golden.py)
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        from make_nn_golden import apply_edit

        apply_edit(str(tmp_path), str(g["xmledit"]))
    if "cellmode" in g.files:  # -cellmode:half on the reference's command line
        return XmlCase(str(tmp_path / "CaseNN"), cellmode=int(g["cellmode"]))
    return XmlCase(str(tmp_path / "CaseNN"))


@pytest.mark.parametrize("name", NN_FT_GOLDENS)
def test_ft_goldens_and_case(name, tmp_path):
    g = load_nn(name)
    assert int(g["floating"]) == 1 and all(("noise_%d" % k) in g.files for k in steps(g))
    x = ft_case(g, tmp_path)
    assert len(x.floatings) == 1 and x.rheology == 2
    # the body sits in the phase-0 layer: its particles replace fluid lattice points
    assert x.floatings[0]["count"] == 343


@pytest.mark.gpu
@pytest.mark.parametrize("name", NN_FT_GOLDENS)
def test_gpu_nn_floating_match_reference_parts(name, tmp_path):
    g = load_nn(name)
    s = gpu(ft_case(g, tmp_path))
    done = 0
    for k in steps(g):
        s.run(k - done)
        done = k
        ref = snapshot(g, k)
        check(by_idp(s.particles()), ref, nn_tol(g, k), k)
        assert abs(s.stats()["time"] - float(ref["time"])) <= 1e-9 * max(1.0, k)


def test_nn_floating_body_moves_in_fixture(tmp_path):
    """The reference integrates the body on the NN interaction's forces: it leaves its start
    position within the fixture's steps (so the GPU test above sees the body dynamics)."""
    g = load_nn(NN_FT_GOLDENS[0])
    f = ft_case(g, tmp_path).floatings[0]
    ref, start = snapshot(g, steps(g)[-1]), snapshot(g, steps(g)[0])
    sel = (ref["idp"] >= f["idbegin"]) & (ref["idp"] < f["idbegin"] + f["count"])
    assert sel.sum() == f["count"]
    assert np.abs(ref["pos"][sel] - start["pos"][sel]).max() > 1e-6
