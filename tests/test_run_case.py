"""Case XML loader + run driver (the callers of the hot path).

Fixtures (tests/golden/make_bi4.py, written by the REFERENCE solver):
  * domains.json — map limits the reference derives from <simulationdomain>, legacy
    IncZ / DomainFixed* and -domain_fixed;
  * sched_*.json / sched_*_last.bi4 — runs on the output schedule (-tmax:0.01 -tout:0.002):
    every PART's header values and the last PART; a restart from the reference's Part_0002.
CPU tests: loader vs the generator and the reference's map limits, refusal of features
this core does not run, the output-time sequence, PART domain limits, the batching of
the driver against a step-by-step loop (fake solver).  GPU tests: the driver vs the
reference's schedules.
"""
import json
import os
import shutil
import sys

import numpy as np
import pytest

from golden_io import by_idp, maxdiff

from dualsphysics_multilayer_amd.case import DamBreakCase
from dualsphysics_multilayer_amd.core import case_derive, read_part
from dualsphysics_multilayer_amd.run import CaseRun, OutputTime, cell_domain_limits, parse_args
from dualsphysics_multilayer_amd.xmlcase import CaseError, XmlCase, parse_pos_value

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bi4")
CASE = os.path.join(FIX, "CaseDambreak")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from make_bi4 import variant_xml  # noqa: E402


def _case_dir(tmp_path, xml_text=None):
    d = tmp_path / "case"
    d.mkdir(exist_ok=True)
    shutil.copy(CASE + ".bi4", d / "CaseDambreak.bi4")
    with open(CASE + ".xml") as fh:
        xml = fh.read()
    (d / "CaseDambreak.xml").write_text(xml_text(xml) if xml_text else xml)
    return str(d / "CaseDambreak")


def test_xml_case_is_the_generated_case():
    x, d = XmlCase(CASE), DamBreakCase(0.05)
    assert x.case_def() == d.case_def()
    for k in ("idp", "pos", "vel", "rhop", "code"):
        assert np.array_equal(getattr(x, k), getattr(d, k)), k
    assert (x.timemax, x.timeout, x.app) == (1.5, 0.01, "gencase_ref")
    s = XmlCase(CASE, step_algorithm=2, tdensity=1)
    assert s.case_def() == DamBreakCase(0.05, step_algorithm=2, tdensity=1).case_def()


def test_restart_case_is_the_part_file():
    h, p = read_part(os.path.join(FIX, "Part_0001.bi4"))
    x = XmlCase(CASE, 1, FIX)
    assert x.time0 == h["timestep"] and x.np == h["npok"] and x.npb == 1182
    assert (x.idp[:1182] < 1182).all() and (x.idp[1182:] >= 1182).all()
    q = by_idp(dict(idp=x.idp, pos=x.pos))
    assert np.array_equal(q["pos"], by_idp(p)["pos"])
    assert x.case_def()["map_realposmin"] == tuple(h["map_posmin"])


@pytest.mark.parametrize("text,ismin,want", [
    ("default", True, (0, 0.0)), ("default - 0.1", True, (2, 0.1)), ("default-10%", True, (3, 10.0)),
    ("-0.05", True, (1, -0.05)), ("default + 50%", False, (3, 50.0)), ("Default+0.3", False, (2, 0.3)),
])
def test_simulationdomain_grammar(text, ismin, want):
    assert parse_pos_value(text, ismin) == want


@pytest.mark.parametrize("text,ismin", [("default+1", True), ("default-1", False), ("5%", True),
                                        ("x1default+1", False), ("default+", False), ("default+1%2", False),
                                        ("abc", True)])
def test_simulationdomain_grammar_errors(text, ismin):
    with pytest.raises(CaseError):
        parse_pos_value(text, ismin)


@pytest.mark.parametrize("var", json.load(open(os.path.join(FIX, "domains.json"))), ids=lambda v: v["name"])
def test_map_limits_are_the_references(var, tmp_path):
    path = _case_dir(tmp_path, lambda xml: variant_xml(xml, var["posmin"], var["posmax"], var["params"]))
    o = parse_args([path] + var["cli"])
    ov = dict(o["overrides"])
    if o["domain_fixed"]:
        ov["domain_fixed"] = o["domain_fixed"]
    cd = XmlCase(path, **ov).case_def()
    assert list(cd["map_realposmin"]) == var["map_posmin"]
    assert list(cd["map_realposmax"]) == var["map_posmax"]


def test_simulationdomain_with_legacy_keys_is_refused(tmp_path):
    path = _case_dir(tmp_path, lambda xml: variant_xml(xml, ["default"] * 3, ["default", "default", "default+1"],
                                                       {"IncZ": "0.5"}))
    with pytest.raises(CaseError, match="not allowed"):
        XmlCase(path)


@pytest.mark.parametrize("edit,match", [
    (lambda x: x.replace('key="Kernel" value="2"', 'key="Kernel" value="3"'), "Kernel choice"),
    # mDBC without a <case>_Normals.nbi4 beside the case (JSph.cpp:1337)
    (lambda x: x.replace("<parameters>", '<parameters>\n<parameter key="Boundary" value="2"/>'), "normal vectors"),
    (lambda x: x.replace("<parameters>", '<parameters>\n<parameter key="Boundary" value="2"/>'
                         '<parameter key="SlipMode" value="2"/>'), "slip mode"),
    (lambda x: x.replace("<parameters>", '<parameters>\n<parameter key="XPeriodicIncY" value="0"/>'), "Periodic"),
    (lambda x: x.replace('<data2d value="false"/>', '<data2d value="true"/>'), "dimension of the case"),
    (lambda x: x.replace("</parameters>", "</parameters>\n<special><wavepaddles/></special>"), "special"),
    (lambda x: x.replace('<fixed mkbound="0" mk="10"', '<moving mkbound="0" mk="10"').replace(
        'count="1182"/>\n<fluid', 'count="1182"/>\n<fluid'), "mobile objects"),
    (lambda x: x.replace('<fixed mkbound="0" mk="10"', '<moving mkbound="0" mk="10"').replace(
        "</constants>", '</constants>\n<motion><objreal ref="0"><begin mov="1" start="0"/>'
        '<mvfile id="1" duration="1"/></objreal></motion>'), "mvfile"),
    (lambda x: x.replace('key="DensityDT" value="2"', 'key="DensityDT" value="7"'), "not valid"),
    (lambda x: x.replace('<parameter key="TimeMax" value="1.5"/>', ''), "TimeMax"),
    (lambda x: x.replace('key="RhopOutMin" value="700"', 'key="RhopOutMin" value="1001"'), "outside"),
])
def test_unsupported_configurations_raise(tmp_path, edit, match):
    with pytest.raises(CaseError, match=match):
        XmlCase(_case_dir(tmp_path, edit))


def test_case_particle_count_must_match(tmp_path):
    path = _case_dir(tmp_path, lambda x: x.replace('count="576"', 'count="575"'))
    with pytest.raises(CaseError):
        XmlCase(path)


@pytest.mark.parametrize("argv,match", [
    (["-cpu"], "GPU"), (["-mdbc_noslip"], "slip mode"), (["-initnorpla:mkbound=0"], "Normals"), (["-cubic"], "Wendland"), (["-viscolamsps:0.01"], "invalid"),
    (["-shifting:sometimes"], "invalid"), (["-sv:vtk"], "not supported"), (["-cellmode:quarter"], "invalid"),
    (["-ddt:4"], "invalid"), (["-bogus"], "not supported"),
])
def test_unsupported_options_raise(argv, match):
    with pytest.raises(CaseError, match=match):
        parse_args([CASE] + argv)


def test_viscosity_and_shifting_options():
    """-viscolamsps:<v> (v <= 0.001, JSphCfgRun.cpp:329-333) and -shifting:<mode>, which
    configures ShiftCoef -2 and ShiftTFS 0 (JSphShifting::ConfigBasic defaults, JSph.cpp:825-835)."""
    ov = parse_args([CASE, "-viscolamsps:1e-6", "-shifting:nobound"])["overrides"]
    assert (ov["tvisco"], ov["visco"]) == (2, float(np.float32(1e-6)))
    assert (ov["shift_mode"], ov["shift_coef"], ov["shift_tfs"]) == (1, -2.0, 0.0)
    assert parse_args([CASE, "-viscoart:0.05"])["overrides"]["tvisco"] == 1


def test_options_mirror_the_reference():
    o = parse_args([CASE, "out", "-gpu:0", "-symplectic", "-ddt:1", "-ddtvalue:0.2", "-tmax:0.01", "-tout:0.002",
                    "-nsteps:5", "-svsteps", "-saveposdouble:1", "-partbegin:3", "somedir", "-rhopout:600:1400",
                    "-cfl:0.1", "-viscoart:0.05", "-sv:binx"])
    ov = o["overrides"]
    assert (o["case"], o["dirout"], o["partbegin"], o["partbegin_dir"], o["nsteps"]) == (CASE, "out", 3, "somedir", 5)
    assert o["svsteps"] and o["nortimes"] and o["saveposdouble"] and o["save"]
    assert ov["step_algorithm"] == 2 and ov["tdensity"] == 1 and ov["cflnumber"] == 0.1
    # JSphCfgRun stores -tmax / -tout / -ddtvalue / -viscoart through float
    assert ov["timemax"] == float(np.float32(0.01)) and ov["timeout"] == float(np.float32(0.002))
    assert ov["ddtvalue"] == float(np.float32(0.2)) and ov["visco"] == float(np.float32(0.05))
    assert (ov["rhopoutmin"], ov["rhopoutmax"]) == (600.0, 1400.0)


@pytest.mark.parametrize("tag", ["verlet", "sym_ddt1", "restart"])
def test_output_times_follow_the_reference_schedule(tag):
    """Consecutive reference PARTs bracket GetNextTime of the earlier one."""
    parts = json.load(open(os.path.join(FIX, f"sched_{tag}.json")))
    ot = OutputTime(float(np.float32(0.002)))
    for a, b in zip(parts, parts[1:]):
        tn = ot.next_time(a["timestep"])
        assert a["timestep"] < tn <= b["timestep"]
        assert b["cpart"] == a["cpart"] + 1


@pytest.mark.parametrize("name", ["sched_verlet_last", "sched_sym_ddt1_last", "sched_restart_last", "Part_0004"])
def test_part_domain_limits_are_the_references(name):
    h, p = read_part(os.path.join(FIX, name + ".bi4"))
    k = case_derive(XmlCase(CASE).case_def())
    npb = int((p["idp"] < 1182).sum())
    assert (p["idp"][:npb] < 1182).all()  # saved in cell order: boundary first
    dmin, dmax = cell_domain_limits(k, p["pos"], npb)
    assert dmin == h["domain_min"] and dmax == h["domain_max"]


class _FakeSolver:
    """Stands in for SphGpuSingle in the batching test: dt from a fixed sequence; a
    Symplectic step advances by the dt of the step before (DtIni first)."""

    def __init__(self, dts, sym=False, dtini=0.0, np_=1758, npb=1182):
        self.dts, self.sym, self.i, self.t, self.np, self.npb = dts, sym, 0, 0.0, np_, npb
        self.dtpre = dtini
        self.calls = []

    def advance(self):
        if self.sym:
            self.t += self.dtpre
            self.dtpre = self.dts[self.i]
        else:
            self.t += self.dts[self.i]
        self.i += 1

    def run(self, n):
        self.calls.append(n)
        for _ in range(n):
            self.advance()

    def stats(self):
        return dict(time=self.t, nstep=self.i, np=self.np, npb=self.npb, nout=0, sym_dtpre=self.dtpre, error_flags=0)

    def close(self):
        pass


@pytest.mark.parametrize("sym", [False, True])
def test_batched_driver_saves_where_a_step_loop_saves(monkeypatch, sym):
    case = XmlCase(CASE, timemax=0.05, timeout=0.004, step_algorithm=2 if sym else 1)
    cap = case.dt_cap()
    dtini = case_derive(case.case_def())["dtini"]
    rng = np.random.default_rng(7)
    dts = list(cap * rng.uniform(0.55, 1.0, 400) / (1 + 1e-9))
    # reference loop, one step at a time (JSphGpuSingle.cpp:849-883)
    ref = _FakeSolver(dts, sym, dtini)
    ot, nstep, want = OutputTime(case.timeout), 0, [(0, 0.0, 0)]
    tnext, part = ot.next_time(0.0), 1
    while ref.t < case.timemax:
        ref.advance()
        if ref.t >= tnext:
            want.append((part, ref.t, nstep))
            part += 1
            tnext = ot.next_time(ref.t)
        nstep += 1
    fake = _FakeSolver(dts, sym, dtini)
    monkeypatch.setattr("dualsphysics_multilayer_amd.run.SphGpuSingle", lambda c, device=0: fake)
    r = CaseRun(case, "unused", save=False, log=lambda s: None)
    got = [(p["cpart"], p["time"], p["step"]) for p in r.run()]
    assert got == want
    assert r.nsteps == nstep and max(fake.calls) > 3 and len(fake.calls) < nstep / 2


# ---- GPU: the driver vs the reference's schedules ---------------------------------------------
def _run_cli(tmp_path, argv):
    from dualsphysics_multilayer_amd.run import main

    out = str(tmp_path / "out")
    assert main([CASE, out] + argv + ["-tmax:0.01", "-tout:0.002", "-saveposdouble:1", "-sv:binx"]) == 0
    return out


def _check_schedule(out, tag, tol):
    ref = json.load(open(os.path.join(FIX, f"sched_{tag}.json")))
    names = sorted(f for f in os.listdir(out) if f.startswith("Part_") and f.endswith(".bi4"))
    assert len(names) == len(ref)
    for f, r in zip(names, ref):
        h, _ = read_part(os.path.join(out, f))
        assert (h["cpart"], h["step"], h["npok"], h["nout"]) == (r["cpart"], r["step"], r["npok"], r["nout"]), f
        assert abs(h["timestep"] - r["timestep"]) <= 1e-8, f
        assert h["domain_min"] == r["domain_min"] and h["domain_max"] == r["domain_max"], f
        assert abs(h["symplectic_dtpre"] - r["symplectic_dtpre"]) <= 1e-9
    _, got = read_part(os.path.join(out, names[-1]))
    _, exp = read_part(os.path.join(FIX, f"sched_{tag}_last.bi4"))
    got, exp = by_idp(got), by_idp(exp)
    assert np.array_equal(got["idp"], exp["idp"])
    for k, t in zip(("pos", "vel", "rhop"), tol):
        assert maxdiff(got, exp, k) <= t, (k, maxdiff(got, exp, k))


TOL20 = (1e-7, 5e-5, 1e-2)  # test_gpu_parity.tol(20): 10x the noise floor at 20 steps


@pytest.mark.gpu
def test_gpu_run_on_schedule_verlet(tmp_path):
    _check_schedule(_run_cli(tmp_path, []), "verlet", TOL20)


@pytest.mark.gpu
def test_gpu_run_on_schedule_symplectic_ddt1(tmp_path):
    _check_schedule(_run_cli(tmp_path, ["-symplectic", "-ddt:1"]), "sym_ddt1", TOL20)


@pytest.mark.gpu
def test_gpu_restart_on_schedule(tmp_path):
    src = tmp_path / "src"
    src.mkdir()
    shutil.copy(os.path.join(FIX, "sched_verlet_Part_0002.bi4"), src / "Part_0002.bi4")
    _check_schedule(_run_cli(tmp_path, ["-partbegin:2", str(src)]), "restart", TOL20)
