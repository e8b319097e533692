"""The dt and viscosity options of <execution><parameters> (JSph::LoadConfigParameters,
JSph.cpp:619-622,697-707): DtFixed (a constant dt), DtFixedFile (dt(t) in ms, JDsFixedDt),
ViscoTime (Visco(t), JDsViscoInput, set at every step's TimeStep, JSphCpuSingle.cpp:1092) and
DtAllParticles (VelMax over every particle, JSphCpu.cpp:475).

Fixtures (tests/golden/make_dtopt_case.py): the REFERENCE DualSPHysics v5.2 CPU solver run on
gencase_ref's dam break / genflume_ref's flume with the option added to the case XML, its
PARTs and the fast-math vs strict-build noise floor.  CPU tests pin the case loader (data
files, the dt cap of the run driver); GPU tests run the case files through the C-ABI and
hold every kept PART to 10x the reference's own noise floor and its times to 1e-8 s per step.
"""
import os

import numpy as np
import pytest

from golden_io import maxdiff

from dualsphysics_multilayer_amd.xmlcase import XmlCase

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "bi4")
VARIANTS = ("verlet_ddt2_dtfixed", "symplectic_ddt1_dtfixedfile", "verlet_ddt2_viscotime",
            "flume_verlet_ddt2_dtallparticles", "verlet_ddt2_dtfixedfile_unordered", "verlet_ddt2_viscotime_unordered")
FLOOR = (2e-10, 2e-7, 2.5e-3)  # pos m, vel m/s, rho kg/m3 (as tests/test_ext.py)


def _dir(v):
    return os.path.join(FIX, "dtopt_" + v)


def _case(v):
    d = _dir(v)
    name = "CaseFlume" if v.startswith("flume") else "CaseDambreak"
    return XmlCase(os.path.join(d, name))


def _ref(v):
    return np.load(os.path.join(_dir(v), "ref.npz"))


def _kept(g):
    return sorted(int(k[1:].split("_")[0]) for k in g.files if k.startswith("s") and k.endswith("_idp"))


def _tol(g, k):
    n = g["noise_%d" % k]
    return tuple(max(10.0 * float(n[i]), FLOOR[i]) for i in range(3))


# ---- case loader (CPU) ------------------------------------------------------------------------
def test_loader_reads_the_dt_options():
    x = _case("verlet_ddt2_dtfixed")
    assert x.dtfixed == 2e-4 and x.dtfixed_table is None and x.case_def()["dtfixed"] == 2e-4
    x = _case("symplectic_ddt1_dtfixedfile")
    assert x.dtfixed == 0 and np.array_equal(x.dtfixed_table, [[0, 0.08], [0.006, 0.22], [1, 0.22]])
    assert x.dt_cap() == pytest.approx(0.22e-3, rel=1e-8)  # the run driver's batch bound
    x = _case("verlet_ddt2_viscotime")
    assert np.array_equal(x.visco_table, [[0, 0.01], [0.004, 0.6], [1, 0.6]])
    x = _case("flume_verlet_ddt2_dtallparticles")
    assert x.dtallparticles == 1 and x.case_def()["dtallparticles"] == 1


def test_loader_refuses_dtfixed_with_a_file(tmp_path):
    from dualsphysics_multilayer_amd.xmlcase import CaseError

    d = _dir("symplectic_ddt1_dtfixedfile")
    for f in os.listdir(d):
        if f != "ref.npz":
            open(tmp_path / f, "wb").write(open(os.path.join(d, f), "rb").read())
    xml = (tmp_path / "CaseDambreak.xml").read_text()
    (tmp_path / "CaseDambreak.xml").write_text(xml.replace("</parameters>", '<parameter key="DtFixed" '
                                                                            'value="1e-4"/></parameters>'))
    with pytest.raises(CaseError, match="cannot be used at the same time"):
        XmlCase(str(tmp_path / "CaseDambreak"))


@pytest.mark.parametrize("v", VARIANTS)
def test_fixtures_present(v):
    g = _ref(v)
    assert _kept(g) and all(("noise_%d" % k) in g.files for k in _kept(g))


def test_reference_used_the_fixed_dt():
    """The fixtures show each option at work: every Verlet step of DtFixed is 2e-4; the
    DtFixedFile steps follow the table (ms) from the second step on (the first Symplectic
    step runs with DtIni)."""
    dt = np.diff(_ref("verlet_ddt2_dtfixed")["times"])
    assert np.allclose(dt, 2e-4, rtol=0, atol=1e-15)
    g = _ref("symplectic_ddt1_dtfixedfile")
    t, dt = g["times"], np.diff(g["times"])
    # a Symplectic step runs with SymplecticDtPre: the table at the previous step's TimeStep
    assert np.abs(dt[1:] - np.interp(t[:-2], [0, 0.006, 1], [0.08e-3, 0.22e-3, 0.22e-3])).max() < 1e-17


def _walk(T, V, ts):
    """JDsFixedDt::GetDt's walk (JDsFixedDt.cpp:111-124) with its persistent Position."""
    pos, out = 0, []
    for t in ts:
        tini, tnext = T[pos], (T[pos + 1] if pos + 1 < len(T) else T[pos])
        while tnext < t and pos + 2 < len(T):
            tini, tnext = tnext, T[pos + 2]
            pos += 1
        out.append(V[pos] if t <= tini else V[pos + 1] if t >= tnext
                   else (t - tini) / (tnext - tini) * (V[pos + 1] - V[pos]) + V[pos])
    return np.array(out)


def test_reference_walks_unordered_rows():
    """A DtFixedFile with rows out of time order: the reference takes it, and past the
    out-of-order row its dt follows the walk from the row of the last lookup (0.15 -> 0.3 ms
    over [0.003 s, 1 s]), not the rows sorted by time; the loader keeps the file's order."""
    x = _case("verlet_ddt2_dtfixedfile_unordered")
    T, V = x.dtfixed_table[:, 0], x.dtfixed_table[:, 1] / 1000
    assert list(T) == [0, 0.006, 0.003, 1]
    t = _ref("verlet_ddt2_dtfixedfile_unordered")["times"]
    dt = np.diff(t)
    assert np.abs(dt - _walk(T, V, t[:-1])).max() < 1e-17
    o = np.argsort(T, kind="stable")
    assert np.abs(dt - np.interp(t[:-1], T[o], V[o])).max() > 1e-5
    assert list(_case("verlet_ddt2_viscotime_unordered").visco_table[:, 0]) == [0, 0.004, 0.002, 1]


# ---- GPU ----------------------------------------------------------------------------------------
def _run_check(s, g, k0=0):
    done = k0
    for k in _kept(g):
        s.run(k - done)
        done = k
        got = s.particles()
        o = np.argsort(got["idp"], kind="stable")
        got = {q: got[q][o] for q in ("idp", "pos", "vel", "rhop")}
        ref = {q: g["s%d_%s" % (k, q)] for q in ("idp", "pos", "vel", "rhop")}
        assert np.array_equal(got["idp"], ref["idp"]), "excluded/duplicated particles"
        tp, tv, tr = _tol(g, k)
        assert maxdiff(got, ref, "pos") <= tp, (k, maxdiff(got, ref, "pos"), tp)
        assert maxdiff(got, ref, "vel") <= tv, (k, maxdiff(got, ref, "vel"), tv)
        assert maxdiff(got, ref, "rhop") <= tr, (k, maxdiff(got, ref, "rhop"), tr)
        st = s.stats() if not isinstance(s.stats(), list) else s.stats()[0]
        # the variable dt follows maxima that carry rounding: 1e-8 per step (as test_gpu_slab)
        assert abs(st["time"] - float(g["times"][k])) <= 1e-8 * max(1, k), (k, st["time"], g["times"][k])


@pytest.mark.gpu
@pytest.mark.parametrize("v", VARIANTS)
def test_gpu_matches_reference_parts(v):
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    x, g = _case(v), _ref(v)
    s = SphGpuSingle(x, device=0)
    _run_check(s, g)


@pytest.mark.gpu
@pytest.mark.parametrize("v", ["verlet_ddt2_viscotime", "symplectic_ddt1_dtfixedfile",
                               "verlet_ddt2_dtfixedfile_unordered"])
def test_gpu_slabs_match_reference_parts(v):
    from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition

    x, g = _case(v), _ref(v)
    _run_check(SphSlabGroup(x, slab_partition(x, 2)), g)


@pytest.mark.gpu
@pytest.mark.parametrize("v,off", [("verlet_ddt2_viscotime", {"visco_table": None}),
                                   ("flume_verlet_ddt2_dtallparticles", {"dtallparticles": 0}),
                                   ("symplectic_ddt1_dtfixedfile", {"dtfixed_table": None})])
def test_gpu_option_is_seen(v, off):
    """Each option switched off moves the run off the reference's PART by more than the
    tolerance (the parity tests above would see a core that ignored it)."""
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    x, g = _case(v), _ref(v)
    for a, val in off.items():
        setattr(x, a, val)
    s = SphGpuSingle(x, device=0)
    k = _kept(g)[-1]
    s.run(k)
    got = s.particles()
    o = np.argsort(got["idp"], kind="stable")
    ref = {q: g["s%d_%s" % (k, q)] for q in ("idp", "pos", "vel", "rhop")}
    got = {q: got[q][o] for q in ("idp", "pos", "vel", "rhop")}
    tp, tv, tr = _tol(g, k)
    assert maxdiff(got, ref, "pos") > 10 * tp or maxdiff(got, ref, "vel") > 10 * tv
    # ... and the simulated time by more than the parity bound
    assert abs(s.stats()["time"] - float(g["times"][k])) > 1e-8 * k or v == "verlet_ddt2_viscotime"
