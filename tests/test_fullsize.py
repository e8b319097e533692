"""The BASELINE configurations at their stated sizes (BASELINE.json configs 3-5).

The small reference fixtures pin every formulation; these tests check the numbers the
bench times, at full size:

* cfg2 (1,025,964 particles, Verlet + DDT2) and cfg3 (9,969,118 particles, Symplectic +
  DDT (Molteni) 0.1): the GPU after steps 1, 2 and 10 (cfg2) / 1, 2 and 5 (cfg3) against
  the REFERENCE v5.2 solver run here on the case gencase_ref writes, and cfg3 also against
  the oracle (the C++ restatement of JSphCpu pinned to the reference's PARTs,
  tests/test_oracle_golden.py), at the step tolerances of test_gpu_parity;
* cfg4, wave flume of 4,007,978 particles with a piston, a flap and a floating box, mDBC,
  Verlet + DDT2: the GPU after steps 1, 2 and 10 against the REFERENCE v5.2 solver run here
  on the case genflume_ref writes (PARTs and the body state of PartFloat.fbi4), then 4
  slabs against one domain over 10 steps;
* cfg5, the 3-phase NN wet dam break of 2,015,071 particles: the GPU after 1 step against
  the REFERENCE v5.0 NN solver run here, at 10x the noise floor of its fast-math vs
  strict builds on the same case; per-phase density bounds, determinism and 2 slabs
  against one domain over 5 steps.
The reference binaries are the checkers (oracle/_ref, built from /root/reference by
``make -C oracle``; the strict NN build by ``make -C oracle nnstrict``).
"""
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from golden_io import by_idp, maxdiff, tol

from dualsphysics_multilayer_amd.case import DamBreakCase, WaveFlumeCase, WetDambreakNNCase

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(os.path.dirname(HERE), "oracle", "_ref")
sys.path.insert(0, os.path.join(HERE, "golden"))
CFG3_DP, CFG4_DP, CFG5_DP, CFG5_WIDTH = 0.00205, 0.00265, 0.01, 0.70
THREADS = int(os.environ.get("OMP_NUM_THREADS", "16"))


def _need(*names):
    for n in names:
        if not os.path.exists(os.path.join(REF, n)):
            pytest.skip("oracle/_ref/%s not built" % n)


def _gpu(case):
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    return SphGpuSingle(case, device=0)


def _ref_parts(exe, casepath, nsteps, parts, tmp, tag):
    """Run a reference solver `nsteps` steps saving every PART; the kept parts sorted by idp."""
    from make_golden import load_dump

    out = os.path.join(tmp, "out_" + tag)
    subprocess.check_call([os.path.join(REF, exe), casepath, out, "-nsteps:%d" % nsteps, "-svsteps:1",
                           "-saveposdouble:1", "-sv:binx", "-svres:0", "-ompthreads:%d" % THREADS],
                          stdout=subprocess.DEVNULL, timeout=600)
    res = {}
    fn = os.path.join(tmp, "p.bin")
    for k in parts:
        subprocess.check_call([os.path.join(REF, "partdump_ref"), out, str(k), fn], stdout=subprocess.DEVNULL)
        t, idp, pos, vel, rho = load_dump(fn)
        o = np.argsort(idp, kind="stable")
        res[k] = dict(idp=idp[o], pos=pos[o], vel=vel[o], rhop=rho[o], time=t)
    return res, out


def _check(got, ref, tl, k):
    assert np.array_equal(got["idp"], ref["idp"]), (k, "excluded-particle set differs")
    for q, t in zip(("pos", "vel", "rhop"), tl):
        d = maxdiff(got, ref, q)
        print("step %d %s maxdiff %.3g (tol %.3g)" % (k, q, d, t))
        assert d <= t, (k, q, d, t)


# ---- cfg3 -----------------------------------------------------------------------------------
def test_cfg3_10m_matches_oracle():
    oracle = pytest.importorskip("oracle.pyoracle")
    case = DamBreakCase(CFG3_DP, step_algorithm=2, tdensity=1, celldomfixed=True)
    assert case.np == 9969118
    g, o = _gpu(case), oracle.OracleSolver(case, nthreads=THREADS)
    done = 0
    for k in (1, 2):
        g.run(k - done)
        o.run(k - done)
        done = k
        _check(by_idp(g.particles()), by_idp(o.particles()), tol(k), k)
        assert g.stats()["time"] == pytest.approx(o.stats()["time"], rel=1e-7)
    assert g.stats()["error_flags"] == 0


def _dambreak_vs_reference(dp, step_algorithm, ddt, np_expected, ks=(1, 2)):
    """The dam break of spacing dp as gencase_ref writes it for the reference, loaded by the
    case-file reader; the GPU after the steps `ks` against the REFERENCE v5.2 CPU solver run
    here on the same files (PARTs with double positions), at the step tolerances of
    test_gpu_parity (10x the reference's fast-math noise floor)."""
    _need("gencase_ref", "DualSPHysics5.2CPU_ref", "partdump_ref")
    from dualsphysics_multilayer_amd.xmlcase import XmlCase

    tmp = tempfile.mkdtemp(prefix="dambreak_")
    try:
        subprocess.check_call([os.path.join(REF, "gencase_ref"), repr(dp), tmp, str(step_algorithm), str(ddt), "1.5",
                               "CaseDambreak", "1"], stdout=subprocess.DEVNULL)
        case = XmlCase(os.path.join(tmp, "CaseDambreak"))
        assert case.np == np_expected
        ref, _ = _ref_parts("DualSPHysics5.2CPU_ref", os.path.join(tmp, "CaseDambreak"), max(ks), ks, tmp, "ref")
        g = _gpu(case)
        done = 0
        for k in ks:
            g.run(k - done)
            done = k
            _check(by_idp(g.particles()), ref[k], tol(k), k)
            assert abs(g.stats()["time"] - ref[k]["time"]) <= 1e-9
        assert g.stats()["error_flags"] == 0
    finally:
        shutil.rmtree(tmp)


@pytest.mark.timeout(900)
def test_cfg2_1m_matches_reference():
    """BASELINE cfg2 (1,025,964 particles, Verlet, DDT2) against the reference binary after
    steps 1, 2 and 10."""
    _dambreak_vs_reference(0.0045, 1, 2, 1025964, (1, 2, 10))


@pytest.mark.timeout(1500)
def test_cfg3_10m_matches_reference():
    """BASELINE cfg3 (9,969,118 particles, Symplectic, DDT Molteni) against the reference binary
    after steps 1, 2 and 5."""
    _dambreak_vs_reference(CFG3_DP, 2, 1, 9969118, (1, 2, 5))


# ---- cfg4 -----------------------------------------------------------------------------------
def _flume_tol(step):
    """10x the reference's noise floor on the flume (tests/test_bodies.py _tol)."""
    return (1.4e-8, 2.2e-5, 1e-2) if step <= 1 else (2e-7, 6e-5, 1e-2)


def test_cfg4_4m_flume_matches_reference():
    _need("genflume_ref", "DualSPHysics5.2CPU_ref", "partdump_ref", "ftdump_ref")
    from dualsphysics_multilayer_amd.xmlcase import XmlCase
    from make_flume_case import load_ft

    tmp = tempfile.mkdtemp(prefix="cfg4_")
    try:
        subprocess.check_call([os.path.join(REF, "genflume_ref"), repr(CFG4_DP), tmp, "1", "2", "1.0", "CaseFlume", "2"],
                              stdout=subprocess.DEVNULL)
        case = XmlCase(os.path.join(tmp, "CaseFlume"))
        assert case.np == 4007978 and case.np == WaveFlumeCase(CFG4_DP, tboundary=2).np
        ks = (1, 2, 10)
        ref, out = _ref_parts("DualSPHysics5.2CPU_ref", os.path.join(tmp, "CaseFlume"), max(ks), ks, tmp, "ref")
        subprocess.check_call([os.path.join(REF, "ftdump_ref"), out, os.path.join(tmp, "ft.bin")],
                              stdout=subprocess.DEVNULL)
        _, fc, fv, fw = load_ft(os.path.join(tmp, "ft.bin"))
        g = _gpu(case)
        done = 0
        for k in ks:
            g.run(k - done)
            done = k
            _check(by_idp(g.particles()), ref[k], _flume_tol(k), k)
            assert abs(g.stats()["time"] - ref[k]["time"]) <= 1e-9
            b = g.floatings()[0]
            # body state after step k (PartFloat.fbi4 item k): center, fvel, fomega
            assert np.abs(np.array(b["center"]) - fc[k, 0]).max() <= 2e-8
            assert np.abs(np.array(b["fvel"]) - fv[k, 0]).max() <= 3.4e-6
            assert np.abs(np.array(b["fomega"]) - fw[k, 0]).max() <= 3.9e-6
    finally:
        shutil.rmtree(tmp)


def test_cfg4_4m_flume_slabs_match_one_domain():
    """4 slabs (the BASELINE's 4 GPUs, here on one) against one domain over 10 steps: same
    particles, states within the 20-step tolerance, the same body state, no errors."""
    from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition

    case = WaveFlumeCase(CFG4_DP, tboundary=2)
    one = _gpu(case)
    grp = SphSlabGroup(case, slab_partition(case, 4))
    one.run(10)
    grp.run(10)
    p1, pg = by_idp(one.particles()), grp.particles()
    _check(pg, p1, _flume_tol(10), 10)
    assert all(st["error_flags"] == 0 for st in grp.stats()) and one.stats()["error_flags"] == 0
    assert np.isfinite(pg["pos"]).all() and np.isfinite(pg["vel"]).all()
    b1, bg = one.floatings()[0], grp.floatings()[0]
    for q, t in (("center", 2e-8), ("fvel", 3.4e-6), ("fomega", 3.9e-6)):
        assert np.abs(np.array(b1[q]) - np.array(bg[q])).max() <= t, q


# ---- cfg5 -----------------------------------------------------------------------------------
NN_FLOOR = (2e-10, 2e-8, 2.5e-3)


def test_cfg5_2m_nn_matches_reference():
    """Steps 1 and 3 of the 2M NN case against the reference v5.0 NN solver, at 10x the
    fast-math vs strict difference of the reference itself on this case at the same step
    (with few-ulp floors)."""
    _need("gennn_ref", "DualSPHysics5.0NN_CPU_ref", "partdump_ref")
    strict = os.path.exists(os.path.join(REF, "DualSPHysics5.0NN_CPU_strict"))
    from dualsphysics_multilayer_amd.xmlcase import XmlCase

    tmp = tempfile.mkdtemp(prefix="cfg5_")
    try:
        subprocess.check_call([os.path.join(REF, "gennn_ref"), repr(CFG5_DP), tmp, repr(CFG5_WIDTH), "1", "5", "CaseNN"],
                              stdout=subprocess.DEVNULL)
        case = XmlCase(os.path.join(tmp, "CaseNN"))
        assert case.np == WetDambreakNNCase(CFG5_DP, width=CFG5_WIDTH).np == 2015071
        ref, _ = _ref_parts("DualSPHysics5.0NN_CPU_ref", os.path.join(tmp, "CaseNN"), 3, (1, 3), tmp, "ref")
        g = _gpu(case)
        done = 0
        for k in (1, 3):
            if strict:
                if k == 1:
                    refs, _ = _ref_parts("DualSPHysics5.0NN_CPU_strict", os.path.join(tmp, "CaseNN"), 3, (1, 3), tmp,
                                         "strict")
                noise = [maxdiff(ref[k], refs[k], q) for q in ("pos", "vel", "rhop")]
            else:  # the noise floor of the 20k-particle fixture (tests/golden/nn_sym_lam_dp0.02.npz):
                # step 1, or step 10 for step 3
                noise = list(np.load(os.path.join(HERE, "golden", "nn_sym_lam_dp0.02.npz"))["noise_%d" % (1 if k == 1
                                                                                                          else 10)])
            tl = tuple(max(10.0 * float(noise[i]), NN_FLOOR[i]) for i in range(3))
            g.run(k - done)
            done = k
            _check(by_idp(g.particles()), ref[k], tl, k)
            assert abs(g.stats()["time"] - ref[k]["time"]) <= 1e-9 * k
    finally:
        shutil.rmtree(tmp)


def test_cfg5_2m_nn_properties_and_slabs():
    """20 steps of the 2M NN case: count kept, finite state, each phase's density within
    [0.9, 1.1] x its rest density, bitwise determinism; 2 slabs (the BASELINE's 2 GPUs, here
    on one) against one domain after 5 steps at the NN fixtures' 10-step tolerance."""
    from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition

    case = WetDambreakNNCase(CFG5_DP, width=CFG5_WIDTH)
    a, b = _gpu(case), _gpu(case)
    a.run(20)
    b.run(20)
    pa, pb = a.particles(), b.particles()
    for q in ("idp", "pos", "vel", "rhop"):
        assert np.array_equal(pa[q], pb[q]), q
    st = a.stats()
    assert st["np"] == case.np and st["nout"] == 0 and st["error_flags"] == 0
    assert np.isfinite(pa["pos"]).all() and np.isfinite(pa["vel"]).all()
    p = by_idp(pa)
    code = case.code[p["idp"]]
    for k, ph in enumerate(case.phases):
        m = (code & 0x1800) == 0x1800
        m &= (code & 0x7ff) == k
        r = p["rhop"][m]
        assert (r > 0.9 * ph["rho"]).all() and (r < 1.1 * ph["rho"]).all(), (k, r.min(), r.max())
    one = _gpu(case)
    grp = SphSlabGroup(case, slab_partition(case, 2))
    one.run(5)
    grp.run(5)
    _check(grp.particles(), by_idp(one.particles()), (1e-8, 1e-5, 1e-2), 5)
