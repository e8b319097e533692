"""Moving boundaries and floating bodies.

Reference: JSph::CalcMotion / JMotion::ProcesTimeSimple + JSphCpu::RunMotion (moving
objects, JSph.cpp:2308, JMotion.cpp:347-366, JMotionObj.cpp:368-580, JSphCpu.cpp:1692-1789)
and JSphCpuSingle::RunFloating (RigidAlgorithm=1, JSphCpuSingle.cpp:748-1010); floating
particles in the interaction (JSphCpu.cpp:656-705) and in the updates (JSphCpu.cpp:1352,
1475, 1577).

Fixtures (written by the REFERENCE solver, tests/golden/make_flume_case.py): a wave flume
with a piston (mvrectsinu), a flap (wait -> mvrotsinu about the hinge line), a floating
box and still water; PART snapshots + the floating-body state of every PART
(PartFloat.fbi4).  CPU tests pin the case loader and the motion semantics (units, the
wait -> rotation chain) against the moving particles of the reference PARTs with a small
restatement of the two movements; GPU tests run the HIP path through the C-ABI against
the reference PARTs and body states.
"""
import math
import os

import numpy as np
import pytest

from golden_io import by_idp, maxdiff

from dualsphysics_multilayer_amd.xmlcase import CaseError, XmlCase

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "bi4")
VARIANTS = ["verlet_ddt2", "symplectic_ddt1_mdbc"]
# mDBC on the floating box too (its outer layer has normals: UseNormalsFt, JSph.cpp:1301-1306;
# the normals turned with the body, JSphCpuSingle.cpp:988-999), and MDBCCorrector=1 (mDBC also
# before the Symplectic corrector, JSphCpuSingle.cpp:525)
FT_VARIANTS = ["verlet_ddt2_mdbc_ftnor", "symplectic_ddt1_mdbc_ftnor", "symplectic_ddt1_mdbc_corr"]


def _case(variant):
    return XmlCase(os.path.join(FIX, "flume_" + variant, "CaseFlume"))


def _ref(variant):
    return np.load(os.path.join(FIX, "flume_" + variant, "ref.npz"))


def _snap(g, k):
    return {q: g["s%d_%s" % (k, q)] for q in ("idp", "pos", "vel", "rhop")}


def _kept(g):
    return sorted(int(k[1:].split("_")[0]) for k in g.files if k.startswith("s") and k.endswith("_idp"))


# ---- case loader (CPU) ---------------------------------------------------------------------
@pytest.mark.parametrize("variant", VARIANTS + FT_VARIANTS)
def test_flume_case_blocks_and_codes(variant):
    x = _case(variant)
    assert x.has_bodies and x.case_nmoving == 2 * 16 * 11 and x.case_nfloat == 125
    assert x.npb == x.case_nfixed + x.case_nmoving
    code = x.code
    # JSphMk::Config: moving blocks 0,1 and floating block 0 (JSphMk.cpp:108-114)
    assert set(np.unique(code[: x.npb])) == {0x0, 0x800, 0x801}
    assert set(np.unique(code[x.npb:])) == {0x1000, 0x1800}
    assert (x.idp[: x.npb] < x.case_npb).all() and (x.idp[x.npb:] >= x.case_npb).all()
    f = x.floatings[0]
    assert f["idbegin"] == x.case_npb and f["count"] == 125
    assert f["massbody"] == pytest.approx(500.0 * 125 * 0.025 ** 3)
    m = x.motion
    assert m["nobj"] == 2 and [v["type"] for v in m["movs"]] == [6, 1, 7]
    assert m["movs"][1]["duration"] == float(np.float32(0.004))  # GetAttributeFloat


@pytest.mark.parametrize("variant", FT_VARIANTS)
def test_floating_normals_and_corrector_loaded(variant):
    """The loader takes the floating box's normals (its outer layer: 98 of 125 particles) and
    MDBCCorrector (JSph.cpp:639,783) into the case definition."""
    x = _case(variant)
    nor = x.boundnormal
    fl = (x.idp >= x.case_npb) & (x.idp < x.case_nbound)
    assert (np.abs(nor[fl]).sum(axis=1) > 0).sum() == 125 - 27
    assert not nor[x.idp >= x.case_nbound].any()
    assert x.case_def()["mdbc_corrector"] == (1 if variant.endswith("_corr") else 0)


def test_unsupported_body_features_refused(tmp_path):
    src = os.path.join(FIX, "flume_verlet_ddt2")
    xml = open(os.path.join(src, "CaseFlume.xml")).read()
    import shutil

    def variant(edit):
        d = tmp_path / ("c%d" % len(list(tmp_path.iterdir())))
        d.mkdir()
        shutil.copy(os.path.join(src, "CaseFlume.bi4"), d / "CaseFlume.bi4")
        (d / "CaseFlume.xml").write_text(edit(xml))
        return str(d / "CaseFlume")

    with pytest.raises(CaseError, match="RigidAlgorithm"):
        XmlCase(variant(lambda s: s.replace('key="RigidAlgorithm" value="1"', 'key="RigidAlgorithm" value="2"')))
    with pytest.raises(CaseError, match="file not found"):  # a table file the case does not have
        XmlCase(variant(lambda s: s.replace("</floating>", '<linearvel file="vel.csv"/></floating>')))
    with pytest.raises(CaseError, match="not found 'axisp1'"):  # an mvcir needs its axis (tests/test_motion.py)
        XmlCase(variant(lambda s: s.replace("<wait ", "<mvcir ")))
    with pytest.raises(CaseError, match="mobile objects"):
        XmlCase(variant(lambda s: s.replace('<objreal ref="1">', '<objreal ref="3">')))


def _rot_y(p, hinge_x, ang_deg):
    """Rotation about the line from (hinge_x, 0, 0) to (hinge_x, 1, 0) (JMatrix4::MatrixRot:
    x' = c x - s z, z' = s x + c z)."""
    a = math.radians(ang_deg)
    c, s = math.cos(a), math.sin(a)
    x, z = p[:, 0] - hinge_x, p[:, 2]
    return np.stack([hinge_x + c * x - s * z, p[:, 1], s * x + c * z], axis=1)


@pytest.mark.parametrize("variant", VARIANTS)
def test_motion_semantics_match_reference_parts(variant):
    """The parsed program, restated for the piston (x += A sin(phase) increments) and the
    flap (rotation by A sin(2 pi f (t - 0.004)) degrees once the wait ends), reproduces the
    moving particles of the reference PARTs from the reference's own times."""
    x, g = _case(variant), _ref(variant)
    times = g["times"]
    pist = [b for b in x.moving_blocks][0]
    flap = [b for b in x.moving_blocks][1]
    mp, mf = x.motion["movs"][0], x.motion["movs"][2]
    wait = x.motion["movs"][1]["duration"]
    hinge = mf["axisp1"][0]
    p0 = by_idp(dict(idp=x.idp, pos=x.pos))
    for k in _kept(g):
        ref = _snap(g, k)
        t = times[k]
        # piston: the phase accumulates per step; its sum telescopes to A sin(2 pi f t)
        dx = mp["vec2"][0] * math.sin(mp["vec"][0] * 2 * math.pi * t)
        sel = (ref["idp"] >= pist["begin"]) & (ref["idp"] < pist["begin"] + pist["count"])
        exp = p0["pos"][ref["idp"][sel]].copy()
        exp[:, 0] += dx
        assert np.abs(ref["pos"][sel] - exp).max() < 1e-12
        assert np.abs(ref["vel"][sel][:, 1:]).max() == 0
        # flap
        ang = mf["ang2"] * math.sin(mf["ang"] * 2 * math.pi * max(0.0, t - wait))
        sel = (ref["idp"] >= flap["begin"]) & (ref["idp"] < flap["begin"] + flap["count"])
        exp = _rot_y(p0["pos"][ref["idp"][sel]], hinge, ang)
        assert np.abs(ref["pos"][sel] - exp).max() < 1e-11, (k, np.abs(ref["pos"][sel] - exp).max())


# ---- HIP path (GPU) --------------------------------------------------------------------------
def _gpu(case):
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    return SphGpuSingle(case, device=0)


def _tol(step):
    """Per-particle tolerances vs the reference PARTs: 10x the reference's own noise floor
    (the same solver with and without -ffast-math; the mDBC floor of test_mdbc, which the
    floating body does not widen at these step counts)."""
    if step <= 1:
        return 1.4e-8, 2.2e-5, 1e-2
    if step <= 20:
        return 2e-7, 6e-5, 1e-2
    return 2e-6, 2.1e-4, 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS + FT_VARIANTS)
def test_gpu_flume_matches_reference_parts(variant):
    x, g = _case(variant), _ref(variant)
    s = _gpu(x)
    done = 0
    for k in _kept(g):
        s.run(k - done)
        done = k
        ref = _snap(g, k)
        got = by_idp(s.particles())
        assert np.array_equal(got["idp"], ref["idp"]), "excluded-particle set differs"
        tp, tv, tr = _tol(k)
        # the dt sequence carries the float noise of the maxima (measured 2e-8 relative)
        assert abs(s.stats()["time"] - g["times"][k]) <= 1e-6 * g["times"][k]
        # moving particles: a pure function of the dt sequence (measured <= 2.4e-10 m)
        mv = (ref["idp"] >= x.case_nfixed) & (ref["idp"] < x.case_npb)
        assert np.abs(got["pos"][mv] - ref["pos"][mv]).max() <= 2e-9
        assert np.abs(got["vel"][mv] - ref["vel"][mv]).max() <= 1e-5
        for q, t in (("pos", tp), ("vel", tv), ("rhop", tr)):
            assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS + FT_VARIANTS)
def test_gpu_floating_body_matches_reference(variant):
    """Body state after every step vs PartFloat.fbi4 (center, fvel, fomega).  Measured on
    MI355X: center <= 2e-8 m, fvel <= 3.4e-6 m/s (|fvel| up to 0.12), fomega <= 3.9e-6
    rad/s (|fomega| up to 5e-3) over 60-100 steps."""
    x, g = _case(variant), _ref(variant)
    s = _gpu(x)
    n = int(g["meta"][3])
    worst = np.zeros(3)
    for k in range(1, n + 1):
        s.run(1)
        b = s.floatings()[0]
        dc = np.abs(b["center"] - g["ft_center"][k, 0]).max()
        dv = np.abs(b["fvel"] - g["ft_fvel"][k, 0]).max()
        dw = np.abs(b["fomega"] - g["ft_fomega"][k, 0]).max()
        worst = np.maximum(worst, [dc, dv, dw])
    vscale = np.abs(g["ft_fvel"]).max()
    wscale = np.abs(g["ft_fomega"]).max()
    assert worst[0] <= 1e-7, worst
    assert worst[1] <= 2e-3 * vscale + 1e-6, (worst, vscale)
    assert worst[2] <= 2e-2 * wscale + 1e-4, (worst, wscale)


@pytest.mark.gpu
def test_gpu_bodies_deterministic():
    x = _case("verlet_ddt2")
    outs = []
    for _ in range(2):
        s = _gpu(x)
        s.run(15)
        outs.append((by_idp(s.particles()), s.floatings()[0]))
    for q in ("pos", "vel", "rhop"):
        assert np.array_equal(outs[0][0][q], outs[1][0][q])
    assert np.array_equal(outs[0][1]["center"], outs[1][1]["center"])


@pytest.mark.gpu
@pytest.mark.parametrize("variant,nslabs", [("verlet_ddt2", 3), ("symplectic_ddt1_mdbc", 2),
                                            ("verlet_ddt2_mdbc_ftnor", 3), ("symplectic_ddt1_mdbc_corr", 2)])
def test_gpu_bodies_on_slabs_match_reference(variant, nslabs):
    """Moving boundaries, the floating body (force sums added over the slabs) and mDBC on
    the x-slab decomposition (in-process slabs on one GPU: the same pack / exchange /
    reduce code as RCCL) vs the reference PARTs and body states."""
    from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition

    x, g = _case(variant), _ref(variant)
    grp = SphSlabGroup(x, slab_partition(x, nslabs))
    done = 0
    for k in _kept(g):
        grp.run(k - done)
        done = k
        got, ref = grp.particles(), _snap(g, k)
        assert np.array_equal(got["idp"], ref["idp"]), "excluded/duplicated particles"
        for q, t in zip(("pos", "vel", "rhop"), _tol(k)):
            assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))
        b = grp.floatings()[0]
        assert np.abs(b["center"] - g["ft_center"][k, 0]).max() <= 1e-7
        assert np.abs(b["fvel"] - g["ft_fvel"][k, 0]).max() <= 2e-3 * np.abs(g["ft_fvel"]).max() + 1e-6


@pytest.mark.parametrize("variant,kw", [("verlet_ddt2", dict()),
                                        ("symplectic_ddt1_mdbc", dict(step_algorithm=2, tdensity=1, tboundary=2)),
                                        ("verlet_ddt2_mdbc_ftnor", dict(tboundary=2, ftnormals=True)),
                                        ("symplectic_ddt1_mdbc_corr", dict(step_algorithm=2, tdensity=1, tboundary=2,
                                                                           ftnormals=True, mdbc_corrector=1))])
def test_product_flume_generator_is_the_reference_case(variant, kw):
    """case.py WaveFlumeCase (the bench's cfg4 generator) == the case genflume_ref wrote
    for the reference, bit for bit: particles, codes, normals, constants, motion program
    and floating body."""
    from dualsphysics_multilayer_amd.case import WaveFlumeCase

    w, x = WaveFlumeCase(0.025, **kw), _case(variant)
    assert w.case_def() == x.case_def()
    for q in ("idp", "pos", "vel", "rhop", "code"):
        assert np.array_equal(getattr(w, q), getattr(x, q)), q
    assert w.motion == x.motion
    assert w.floatings == x.floatings
    if kw.get("tboundary") == 2:
        assert np.array_equal(w.boundnormal, x.boundnormal)


def _moved_case(x, nsteps, cellmode):
    """The case with the particle state of the tiled solver after nsteps (bodies in motion,
    densities off the initial hydrostatic lattice), so an interaction has physical ar/ace
    instead of the t=0 round-off of a balanced lattice."""
    import copy

    y = copy.copy(x)
    y.cellmode = cellmode
    s = _gpu(y)
    s.run(nsteps)
    p = by_idp(s.particles())
    assert np.array_equal(p["idp"], np.sort(x.idp))
    row = np.searchsorted(p["idp"], x.idp)
    y.pos, y.vel, y.rhop = p["pos"][row].copy(), p["vel"][row].copy(), p["rhop"][row].copy()
    return y


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("cellmode", [1, 2])
def test_gpu_tiled_floating_interaction_matches_per_particle_kernel(variant, cellmode, monkeypatch):
    """The floating (FT) instantiation of the LDS-tiled kernel (mass-scaled records, DDT
    rules of floating p1/p2; CellMode full and half) vs the one-lane-per-particle kernel on
    the same state: the flume after 6 steps (fluid around and below the moving box, the
    box's own particles as p1), both within 2e-4 of max|ar| / max|ace| (float rounding of
    different summation orders and fast intrinsics)."""
    x = _moved_case(_case(variant), 6, cellmode)
    monkeypatch.setenv("SPH_INTERACTION", "simple")
    ref = _gpu(x)
    monkeypatch.delenv("SPH_INTERACTION")
    til = _gpu(x)
    for s in (ref, til):
        s.Interaction_Forces(1 if x.step_algorithm == 1 else 2)
    a, b = til.interaction(), ref.interaction()
    assert np.array_equal(til.particles()["idp"], ref.particles()["idp"])
    flt = (til.particles()["code"] & 0x1800) == 0x1000
    assert flt.sum() == x.case_nfloat
    for q in ("ar", "ace"):
        scale = np.abs(b[q]).max()
        assert np.abs(a[q] - b[q]).max() <= 2e-4 * scale, (q, np.abs(a[q] - b[q]).max(), scale)
        assert np.abs(a[q][flt] - b[q][flt]).max() <= 2e-4 * np.abs(b[q][flt]).max() + 1e-6, q


@pytest.mark.gpu
def test_gpu_run_driver_flume_matches_reference(tmp_path):
    """The flume case through the reference's command line (run driver): PART 10 vs the
    reference's PART 10 (moving/floating counts in the header)."""
    from dualsphysics_multilayer_amd.core import read_part
    from dualsphysics_multilayer_amd.run import main

    case = os.path.join(FIX, "flume_verlet_ddt2", "CaseFlume")
    out = str(tmp_path / "out")
    assert main([case, out, "-nsteps:10", "-svsteps:1", "-saveposdouble:1", "-sv:binx"]) == 0
    h, p = read_part(os.path.join(out, "Part_0010.bi4"))
    assert (h["case_nmoving"], h["case_nfloat"]) == (352, 125)
    got, ref = by_idp(p), _snap(_ref("verlet_ddt2"), 10)
    assert np.array_equal(got["idp"], ref["idp"])
    # PartFloat.fbi4 through the reference's reader (oracle/_ref travels with the tree)
    exe = os.path.join(os.path.dirname(HERE), "oracle", "_ref", "ftdump_ref")
    if os.path.exists(exe):
        import subprocess
        import sys

        sys.path.insert(0, os.path.join(HERE, "golden"))
        from make_flume_case import load_ft

        subprocess.check_call([exe, out, str(tmp_path / "ft.bin")], stdout=subprocess.DEVNULL)
        t, c, v, w = load_ft(str(tmp_path / "ft.bin"))
        g = _ref("verlet_ddt2")
        assert len(t) == 11 and np.abs(c[10, 0] - g["ft_center"][10, 0]).max() <= 1e-7
    for q, t in zip(("pos", "vel", "rhop"), _tol(10)):
        assert maxdiff(got, ref, q) <= t, (q, maxdiff(got, ref, q))


def test_partfloat_file_reads_with_the_reference_reader(tmp_path):
    """PartFloat.fbi4 written by the core (sph_partfloat_write) is read by the reference's
    own JPartFloatBi4Load (oracle/_ref/ftdump_ref): times, centres and velocities."""
    import subprocess

    from dualsphysics_multilayer_amd.core import write_partfloat

    exe = os.path.join(os.path.dirname(HERE), "oracle", "_ref", "ftdump_ref")
    if not os.path.exists(exe):
        pytest.skip("reference tools (oracle/_ref) not built here")
    sys_path = os.path.join(HERE, "golden")
    import sys

    sys.path.insert(0, sys_path)
    from make_flume_case import load_ft

    fl = _case("verlet_ddt2").floatings + [dict(mkbound=4, idbegin=9999, count=27, massbody=0.1, masspart=0.1 / 27)]
    rng = np.random.default_rng(1)
    parts = [dict(cpart=k, step=10 * k, time=0.001 * k,
                  bodies=[dict(center=rng.normal(size=3), fvel=rng.normal(size=3), fomega=rng.normal(size=3),
                               facelin=np.zeros(3), faceang=np.zeros(3)) for _ in fl]) for k in range(4)]
    write_partfloat(str(tmp_path / "PartFloat.fbi4"), fl, parts)
    subprocess.check_call([exe, str(tmp_path), str(tmp_path / "ft.bin")], stdout=subprocess.DEVNULL)
    t, c, v, w = load_ft(str(tmp_path / "ft.bin"))
    assert np.array_equal(t, [p["time"] for p in parts])
    assert np.array_equal(c, np.array([[b["center"] for b in p["bodies"]] for p in parts]))
    assert np.array_equal(v, np.array([[b["fvel"] for b in p["bodies"]] for p in parts], np.float32))
    assert np.array_equal(w, np.array([[b["fomega"] for b in p["bodies"]] for p in parts], np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_gpu_bodies_on_slabs_with_repartition_match_reference(variant):
    """Moving boundaries, the floating box (and mDBC) on 3 slabs re-partitioned every 4 steps
    from an uneven start: the reference PARTs and body states still hold."""
    from dualsphysics_multilayer_amd.core import SphSlabGroup, case_derive

    x, g = _case(variant), _ref(variant)
    ncx = case_derive(x.case_def())["dom_cells"][0]
    # uneven start; the middle slab 2W = 4 columns wide (the narrowest with mDBC)
    grp = SphSlabGroup(x, np.array([0, ncx // 5, ncx // 5 + 4, ncx], np.int32))
    grp.set_repartition(4, 0.3, 0.0)
    done = 0
    for k in _kept(g):
        grp.run(k - done)
        done = k
        got, ref = grp.particles(), _snap(g, k)
        assert np.array_equal(got["idp"], ref["idp"]), "excluded/duplicated particles"
        for q, t in zip(("pos", "vel", "rhop"), _tol(k)):
            assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))
        b = grp.floatings()[0]
        assert np.abs(b["center"] - g["ft_center"][k, 0]).max() <= 1e-7
    assert max(i["repartitions"] for i in grp.slab_info()) >= 1


@pytest.mark.gpu
def test_gpu_mdbc_flap_normals_cross_slab_faces():
    """A fast, wide flap (no wait, 8 Hz, 12 degrees; mDBC, Symplectic): its particles cross
    cell columns within the run.  On 3 slabs whose middle one is the narrowest an mDBC slab
    may be (2W = 4 columns, the flap's initial column its last),
    every crossing flap particle migrates with its turned mDBC normal, and every ghost node's
    support stays inside its slab's grid (no SPH_ERR_UNSUPPORTED halo error); the merged
    state holds the reference PARTs (single-domain tolerance) and the single-domain GPU run."""
    from dualsphysics_multilayer_amd.core import SphSlabGroup, case_derive

    x, g = _case("symplectic_ddt1_mdbc_fastflap"), _ref("symplectic_ddt1_mdbc_fastflap")
    k = case_derive(x.case_def())
    flap = np.where((x.code & 0x1800) == 0x800)[0]
    flap = flap[x.pos[flap, 0] > x.pos[:, 0].mean()]  # the flap, not the piston
    cflap = int((x.pos[flap[0], 0] - k["map_realposmin"][0]) // np.float32(k["scell"]))
    b2 = min(cflap + 1, k["dom_cells"][0] - 2)
    grp = SphSlabGroup(x, np.array([0, b2 - 4, b2, k["dom_cells"][0]], np.int32))
    one = _gpu(x)
    done = 0
    for kk in _kept(g):
        grp.run(kk - done)
        one.run(kk - done)
        done = kk
        got, ref = grp.particles(), _snap(g, kk)
        assert np.array_equal(got["idp"], ref["idp"]), "excluded/duplicated particles"
        for q, t in zip(("pos", "vel", "rhop"), _tol(kk)):
            assert maxdiff(got, ref, q) <= t, (kk, q, maxdiff(got, ref, q))
        p1 = by_idp(one.particles())
        for q, t in zip(("pos", "vel", "rhop"), _tol(kk)):
            assert maxdiff(got, p1, q) <= t, (kk, q, maxdiff(got, p1, q))
    # flap particles did leave their initial column (the hand-over happened)
    fin = grp.particles()["pos"][flap]
    cols = ((fin[:, 0] - k["map_realposmin"][0]) // np.float32(k["scell"])).astype(int)
    assert (cols != cflap).any()
    assert all(st["error_flags"] == 0 for st in grp.stats())


# ---- imposed floating velocities and external forces -----------------------------------------
FTVEL = "verlet_ddt2_ftvel"
# the same kind of tables as a data file (<linearvel file=...>, JLinearValue::LoadFile) and
# with rows out of time order (<angularvel>, <linearforce>), walked as the reference walks them
FTVEL_FILE = "verlet_ddt2_ftvel_file_unordered"


def test_floating_tables_from_file_and_unordered_loaded():
    f = _case(FTVEL_FILE).floatings[0]
    big = np.finfo(np.float64).max
    lv = f["linearvel"]  # the data file, in its row order, "none" -> DBL_MAX
    assert lv.shape == (4, 4) and list(lv[:, 0]) == [0.0, 0.02, 0.006, 0.025]
    assert lv[0, 1] == 0.05 and lv[0, 2] == big and lv[1, 3] == 0.05 and lv[2, 1] == 0.2
    assert list(f["angularvel"][:, 0]) == [0.0, 0.02, 0.008, 0.03]  # XML order kept
    assert list(f["linearforce"][:, 0]) == [0.03, 0.0]


def test_floating_tables_loaded():
    """<linearvel>/<angularvel> (JLinearValue with special values: "none" or a missing
    component -> DBL_MAX, not imposed) and <linearforce>/<angularforce> rows (time, x, y, z)."""
    f = _case(FTVEL).floatings[0]
    big = np.finfo(np.float64).max
    lv = f["linearvel"]
    assert lv.shape == (4, 4) and list(lv[:, 0]) == [0.0, 0.006, 0.02, 0.025]
    assert lv[0, 1] == 0.05 and lv[0, 2] == big and lv[1, 2] == big and lv[2, 3] == 0.05 and lv[3, 3] == big
    assert f["angularvel"][1, 2] == -0.6 and f["angularvel"][1, 1] == big
    assert f["linearforce"][1].tolist() == [0.03, 0.5, 0.2, 1.0]
    assert f["angularforce"].shape == (2, 4)
    assert "linearvel" not in _case("verlet_ddt2").floatings[0]


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [FTVEL, FTVEL_FILE])
def test_gpu_floating_imposed_velocity_matches_reference(variant):
    """The floating box with imposed x/z velocities and y rotation rate over time (free
    components integrated) and external forces/torques (JSphCpuSingle.cpp:874-924): body
    state after every step vs the reference's PartFloat.fbi4 -- imposed components equal the
    reference's to float rounding of the table time --, particles vs the reference PARTs."""
    x, g = _case(variant), _ref(variant)
    s = _gpu(x)
    n = int(g["meta"][3])
    kept = set(_kept(g))
    worst = np.zeros(3)
    for k in range(1, n + 1):
        s.run(1)
        b = s.floatings()[0]
        worst = np.maximum(worst, [np.abs(b["center"] - g["ft_center"][k, 0]).max(),
                                   np.abs(b["fvel"] - g["ft_fvel"][k, 0]).max(),
                                   np.abs(b["fomega"] - g["ft_fomega"][k, 0]).max()])
        if k in kept:
            got, ref = by_idp(s.particles()), _snap(g, k)
            assert np.array_equal(got["idp"], ref["idp"])
            for q, t in zip(("pos", "vel", "rhop"), _tol(k)):
                assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))
    assert worst[0] <= 1e-7, worst
    assert worst[1] <= 2e-3 * np.abs(g["ft_fvel"]).max() + 1e-6, worst
    assert worst[2] <= 2e-3 * np.abs(g["ft_fomega"]).max() + 1e-5, worst
    # the imposed components are the table's values (step 1: TimeStep 0)
    b1 = g["ft_fvel"][1, 0]
    assert b1[0] == np.float32(0.05) and g["ft_fomega"][1, 0][1] == np.float32(0.4)
    if variant == FTVEL_FILE:  # the unordered rows matter: the reference's walk is not a sorted lookup
        srt = _ref(FTVEL)
        assert np.abs(g["ft_fomega"][:, 0, 1] - srt["ft_fomega"][:, 0, 1]).max() > 0


@pytest.mark.gpu
def test_gpu_floating_imposed_velocity_on_slabs():
    """The same case on 2 in-process slabs (every rank evaluates the tables; force sums added
    over the slabs) vs the reference PARTs and body states."""
    from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition

    x, g = _case(FTVEL), _ref(FTVEL)
    grp = SphSlabGroup(x, slab_partition(x, 2))
    done = 0
    for k in _kept(g):
        grp.run(k - done)
        done = k
        got, ref = grp.particles(), _snap(g, k)
        assert np.array_equal(got["idp"], ref["idp"])
        for q, t in zip(("pos", "vel", "rhop"), _tol(k)):
            assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))
        b = grp.floatings()[0]
        assert np.abs(b["center"] - g["ft_center"][k, 0]).max() <= 1e-7
        assert np.abs(b["fvel"] - g["ft_fvel"][k, 0]).max() <= 2e-3 * np.abs(g["ft_fvel"]).max() + 1e-6
