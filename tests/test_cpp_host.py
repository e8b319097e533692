"""The C-ABI driven by a compiled C++ host (tests/cpp/host_loop.cpp): the boundary as a
DualSPHysics-side C++ binding would use it, not through ctypes.

The host loads a dam-break case written by the reference-side generator
(oracle/tools/gencase_ref), derives SphCaseDef as JSph::LoadCaseConfig/LoadCaseParticles
do, runs sph_solver_run and writes reference PART files with sph_part_write; the PARTs
must match the reference solver's own PARTs of that case (tests/golden, 10x its noise
floor) and be readable by the reference's reader."""
import os
import subprocess

import numpy as np
import pytest

from golden_io import by_idp, load, maxdiff, snapshot, tol

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "host_loop.cpp")
EXE = os.path.join(ROOT, "tests", "cpp", "host_loop")
LIBDIR = os.path.join(ROOT, "dualsphysics_multilayer_amd", "lib")
REF = os.path.join(ROOT, "oracle", "_ref")


def build_host(out=EXE):
    """g++ against include/sphcore.h and -lsphcore only (no HIP, no Python)."""
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-I" + os.path.join(ROOT, "include"), SRC,
                           "-L" + LIBDIR, "-lsphcore", "-Wl,-rpath," + LIBDIR, "-o", out])
    return out


def test_host_builds_against_the_c_abi(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "libsphcore.so")):
        pytest.skip("libsphcore.so not built")
    exe = build_host(str(tmp_path / "host_loop"))
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
def test_host_loop_parts_match_reference(tmp_path):
    exe = EXE if os.path.exists(EXE) else build_host(str(tmp_path / "host_loop"))
    g = load("verlet_ddt2_dp0.02")
    subprocess.check_call([os.path.join(REF, "gencase_ref"), "0.02", str(tmp_path), "1", "2", "1.5", "CaseDambreak",
                           "1"], stdout=subprocess.DEVNULL)
    out = tmp_path / "out"
    out.mkdir()
    r = subprocess.run([exe, str(tmp_path / "CaseDambreak"), str(out), "1", "10"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    from dualsphysics_multilayer_amd.core import read_part

    for cpart, k in ((1, 1), (2, 10)):
        hdr, p = read_part(str(out / ("Part_%04u.bi4" % cpart)))
        got, ref = by_idp(p), snapshot(g, k)
        assert np.array_equal(got["idp"], ref["idp"])
        for q, t in zip(("pos", "vel", "rhop"), tol(k)):
            assert maxdiff(got, ref, q) <= t, (k, q, maxdiff(got, ref, q))
        assert hdr["step"] == k and abs(hdr["timestep"] - float(ref["time"])) <= 1e-9 * k
    # the reference's own reader reads the host's PART (partdump_ref links JPartDataBi4)
    dump = tmp_path / "p.bin"
    subprocess.check_call([os.path.join(REF, "partdump_ref"), str(out), "2", str(dump)], stdout=subprocess.DEVNULL)
    assert dump.stat().st_size > 0
