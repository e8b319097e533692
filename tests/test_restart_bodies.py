"""Restart (-partbegin) of cases with floating bodies and mDBC.

The reference restarts a floating body from its state at the PART in PartFloat.fbi4 (center,
fvel, fomega; the angles start again from 0: JSphCpu::InitFloating, JSphCpu.cpp:1885-1905)
and mDBC from the normals of the PART in PartExtra_%04u.bi4 (written every SaveExtraParts-th
PART; JSph::ConfigBoundNormals, JSph.cpp:1308-1316; JDsExtraData.cpp).  Fixtures
(tests/golden/make_flume_restart.py): the wave flume run by the reference to PART k0 (its
files there) and the reference restarted from them (rst.npz: PARTs and body states after).

CPU: the readers against the reference's own files; the writer round trip; the case loader's
restart state.  GPU: the core restarted from the reference's files follows the reference's
restart, and a run of the core that writes its own PartFloat / PartExtra files restarts from
them onto the same reference restart.
"""
import os

import numpy as np
import pytest

from golden_io import by_idp, maxdiff

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "bi4")
VARIANTS = ["verlet_ddt2", "symplectic_ddt1_mdbc_ftnor"]


def _dir(v):
    return os.path.join(FIX, "flumerst_" + v)


def _rst(v):
    return np.load(os.path.join(_dir(v), "rst.npz"))


def _meta(g):
    dp, step, ddt, boundary, k0, n = g["meta"]
    return int(boundary), int(k0), int(n)


def _snap(g, k):
    return {q: g["s%d_%s" % (k, q)] for q in ("idp", "pos", "vel", "rhop")}


def _tol(nsteps):
    """The flume tolerances of tests/test_bodies.py for a run of nsteps from one state."""
    if nsteps <= 1:
        return 1.4e-8, 2.2e-5, 1e-2
    if nsteps <= 20:
        return 2e-7, 6e-5, 1e-2
    return 2e-6, 2.1e-4, 2e-2


@pytest.mark.parametrize("v", VARIANTS)
def test_partfloat_reader_matches_the_reference_restart_state(v):
    """PART k0 of PartFloat.fbi4 (written by the reference's run) read by sph_partfloat_read is
    the state the reference's restart starts from: the first record of its own PartFloat."""
    from dualsphysics_multilayer_amd.core import read_partfloat

    g = _rst(v)
    _, k0, _ = _meta(g)
    st = read_partfloat(os.path.join(_dir(v), "PartFloat.fbi4"), k0, 1)
    assert np.array_equal(st["center"][0], g["ft_center"][0, 0])
    assert np.array_equal(st["fvel"][0], g["ft_fvel"][0, 0])
    assert np.array_equal(st["fomega"][0], g["ft_fomega"][0, 0])
    assert st["time"] == g["ft_time"][0]
    with pytest.raises(Exception, match="not found"):
        read_partfloat(os.path.join(_dir(v), "PartFloat.fbi4"), k0 + 50, 1)


def test_extra_normals_reader_and_writer(tmp_path):
    """PartExtra_0008.bi4 of the reference: the fixed walls' vectors to the ghost node are
    exactly twice the case file's normals (they never turn), floating normals are present
    (UseNormalsFt); the core's writer gives a file that reads back the same and that the
    container rewrite reproduces byte for byte."""
    from dualsphysics_multilayer_amd.core import (bi4_rewrite, read_extra_normals, read_normals,
                                                  write_extra_normals)
    from dualsphysics_multilayer_amd.xmlcase import XmlCase

    d = _dir("symplectic_ddt1_mdbc_ftnor")
    x = XmlCase(os.path.join(d, "CaseFlume"))
    nor, useft = read_extra_normals(os.path.join(d, "PartExtra_0008.bi4"), x.case_nbound, x.case_nfloat)
    assert useft and len(nor) == x.case_nbound
    case_nor = read_normals(os.path.join(d, "CaseFlume_Normals.nbi4")).astype(np.float32)
    fixed = np.arange(x.case_nfixed)
    assert np.array_equal(nor[fixed], case_nor[fixed] * np.float32(2))
    with pytest.raises(Exception, match="CaseNbound"):
        read_extra_normals(os.path.join(d, "PartExtra_0008.bi4"), x.case_nbound + 1, x.case_nfloat)
    fn = str(tmp_path / "PartExtra_0003.bi4")
    write_extra_normals(fn, "test", 3, 30, 0.125, x.case_nbound, x.case_nfloat, nor, True)
    back, ft2 = read_extra_normals(fn, x.case_nbound, x.case_nfloat)
    assert ft2 and np.array_equal(back, nor)
    bi4_rewrite(os.path.join(d, "PartExtra_0008.bi4"), str(tmp_path / "rw.bi4"))
    assert open(str(tmp_path / "rw.bi4"), "rb").read() == open(os.path.join(d, "PartExtra_0008.bi4"), "rb").read()


@pytest.mark.parametrize("v", VARIANTS)
def test_case_loader_restart_state(v):
    """XmlCase with -partbegin: the PART's particles, its time, the bodies' state of that PART
    and (mDBC) the PART's normals, halved for the core (which doubles the case's normals)."""
    from dualsphysics_multilayer_amd.core import read_extra_normals
    from dualsphysics_multilayer_amd.xmlcase import XmlCase

    g = _rst(v)
    boundary, k0, _ = _meta(g)
    d = _dir(v)
    x = XmlCase(os.path.join(d, "CaseFlume"), k0, d)
    assert x.time0 == pytest.approx(float(g["ft_time"][0]), abs=0)
    f = x.floatings[0]
    assert np.array_equal(np.array(f["center"]), g["ft_center"][0, 0])
    assert np.array_equal(np.array(f["linvelini"], np.float32), g["ft_fvel"][0, 0])
    assert np.array_equal(np.array(f["angvelini"], np.float32), g["ft_fomega"][0, 0])
    if boundary == 2:
        nor, _ = read_extra_normals(os.path.join(d, "PartExtra_%04u.bi4" % k0), x.case_nbound, x.case_nfloat)
        bn = x.boundnormal
        sel = x.idp < len(nor)
        assert np.array_equal(bn[sel] * np.float32(2), nor[x.idp[sel]])


def _check_run(s, g, k0, n, x, run_steps):
    for j in range(1, n + 1):
        run_steps(1)
        b = s.floatings()[0]
        assert np.abs(b["center"] - g["ft_center"][j, 0]).max() <= 1e-7, (j, b["center"], g["ft_center"][j, 0])
        vscale, wscale = np.abs(g["ft_fvel"]).max(), np.abs(g["ft_fomega"]).max()
        assert np.abs(b["fvel"] - g["ft_fvel"][j, 0]).max() <= 2e-3 * vscale + 1e-6
        assert np.abs(b["fomega"] - g["ft_fomega"][j, 0]).max() <= 2e-2 * wscale + 1e-4
    got, ref = by_idp(s.particles()), _snap(g, k0 + n)
    assert np.array_equal(got["idp"], ref["idp"])
    assert abs(s.stats()["time"] - float(g["times"][-1])) <= 1e-6 * float(g["times"][-1])
    for q, t in zip(("pos", "vel", "rhop"), _tol(n)):
        assert maxdiff(got, ref, q) <= t, (q, maxdiff(got, ref, q))


@pytest.mark.gpu
@pytest.mark.parametrize("v", VARIANTS)
def test_gpu_restart_from_reference_files_follows_the_reference_restart(v):
    from dualsphysics_multilayer_amd.core import SphGpuSingle
    from dualsphysics_multilayer_amd.xmlcase import XmlCase

    g = _rst(v)
    _, k0, n = _meta(g)
    x = XmlCase(os.path.join(_dir(v), "CaseFlume"), k0, _dir(v))
    s = SphGpuSingle(x, device=0)
    _check_run(s, g, k0, n, x, s.run)
    s.close()


@pytest.mark.gpu
def test_gpu_restart_from_own_files(tmp_path):
    """The run driver to PART k0 with -svextraparts:1 (its own PartFloat.fbi4 and
    PartExtra_%04u.bi4), then restarted from its own files: onto the reference's restart
    within the tolerance of k0 + n steps."""
    from dualsphysics_multilayer_amd.run import main

    v = "symplectic_ddt1_mdbc_ftnor"
    g = _rst(v)
    _, k0, n = _meta(g)
    case = os.path.join(_dir(v), "CaseFlume")
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    assert main([case, a, "-nsteps:%d" % k0, "-svsteps:1", "-saveposdouble:1", "-sv:binx", "-svextraparts:1"]) == 0
    assert os.path.exists(os.path.join(a, "PartExtra_%04u.bi4" % k0))
    assert main([case, b, "-partbegin:%d" % k0, a, "-nsteps:%d" % n, "-svsteps:1", "-saveposdouble:1",
                 "-sv:binx"]) == 0
    from dualsphysics_multilayer_amd.core import read_part

    _, p = read_part(os.path.join(b, "Part_%04u.bi4" % (k0 + n)))
    got, ref = by_idp(p), _snap(g, k0 + n)
    assert np.array_equal(got["idp"], ref["idp"])
    for q, t in zip(("pos", "vel", "rhop"), _tol(k0 + n)):
        assert maxdiff(got, ref, q) <= t, (q, maxdiff(got, ref, q))
