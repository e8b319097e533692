"""PART / case files (.bi4), SURVEY.md §8(f) row 2.

Fixtures (tests/golden/make_bi4.py): files written by the REFERENCE solver and its
case generator, the reference reader's view of a PART, and a reference restart.
  * the container reader/writer reproduces reference files byte for byte;
  * a PART read here equals what the reference's own reader returns;
  * a PART + Part_Head.ibi4 written here is read by the reference reader and the
    reference solver restarts from them exactly as from its own files (needs the
    reference binaries of oracle/_ref: build container only);
  * the GPU solver restarted from a reference PART follows the reference restart.
"""
import filecmp
import os
import shutil
import subprocess

import numpy as np
import pytest

from golden_io import by_idp, maxdiff

from dualsphysics_multilayer_amd.case import DamBreakCase
from dualsphysics_multilayer_amd.core import bi4_rewrite, read_part, write_part, write_part_head

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bi4")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
need_ref = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "DualSPHysics5.2CPU_ref")),
                              reason="reference binaries (oracle/_ref) not built here")


@pytest.mark.parametrize("name", ["CaseDambreak.bi4", "Part_0001.bi4", "Part_0004.bi4", "Part_Head.ibi4",
                                  "restart_Part_0004.bi4"])
def test_container_rewrite_is_byte_identical(name, tmp_path):
    dst = str(tmp_path / name)
    bi4_rewrite(os.path.join(FIX, name), dst)
    assert filecmp.cmp(os.path.join(FIX, name), dst, shallow=False)


def test_read_matches_reference_reader():
    h, p = read_part(os.path.join(FIX, "Part_0001.bi4"))
    ref = np.load(os.path.join(FIX, "part1_ref_reader.npz"))
    q = by_idp(p)
    assert h["npok"] == len(ref["idp"]) and h["cpart"] == 1
    assert h["timestep"] == float(ref["time"])
    for k in ("idp", "pos", "vel", "rhop"):
        assert np.array_equal(q[k], ref[k]), k


def test_case_file_and_header_values():
    h, p = read_part(os.path.join(FIX, "CaseDambreak.bi4"))
    case = DamBreakCase(0.05)
    cd = case.case_def()
    assert (h["case_np"], h["case_nfixed"], h["case_nfluid"]) == (case.np, case.npb, case.np - case.npb)
    assert h["dp"] == cd["dp"] and h["rhop0"] == cd["rhop0"] and h["gamma"] == cd["gamma"]
    # the map limits the solver derived (written into its PARTs) are the case's
    hp, _ = read_part(os.path.join(FIX, "Part_0001.bi4"))
    assert hp["map_posmin"] == list(cd["map_realposmin"]) and hp["map_posmax"] == list(cd["map_realposmax"])
    # the generated lattice is the case file's particle set
    assert np.array_equal(p["idp"], case.idp)
    assert np.array_equal(p["pos"], case.pos)
    assert np.array_equal(p["rhop"], case.rhop)


@pytest.mark.parametrize("pos_double", [1, 0])
def test_write_read_roundtrip(tmp_path, pos_double):
    h, p = read_part(os.path.join(FIX, "Part_0004.bi4"))
    h["pos_double"] = pos_double
    f = str(tmp_path / "Part_0004.bi4")
    write_part(f, h, p)
    h2, p2 = read_part(f)
    for k in ("cpart", "npok", "timestep", "case_np", "dp", "map_posmin", "pos_double"):
        assert h2[k] == h[k], k
    assert np.array_equal(p2["idp"], p["idp"]) and np.array_equal(p2["vel"], p["vel"])
    pos = p["pos"] if pos_double else p["pos"].astype(np.float32).astype(np.float64)
    assert np.array_equal(p2["pos"], pos)


def _restart_header(path):
    h, p = read_part(path)
    h.update(visco_type=1, visco=0.1, viscoboundfactor=1.0, gravity=[0.0, 0.0, -9.81], mkbound=10, mkfluid=0)
    return h, p


@need_ref
def test_reference_reader_reads_our_part(tmp_path):
    h, p = _restart_header(os.path.join(FIX, "Part_0001.bi4"))
    write_part(str(tmp_path / "Part_0001.bi4"), h, p)
    dump = str(tmp_path / "p.bin")
    subprocess.check_call([os.path.join(REF, "partdump_ref"), str(tmp_path), "1", dump], stdout=subprocess.DEVNULL)
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import load_dump

    t, idp, pos, vel, rho = load_dump(dump)
    ref = np.load(os.path.join(FIX, "part1_ref_reader.npz"))
    assert t == float(ref["time"])
    assert np.array_equal(idp, ref["idp"]) and np.array_equal(pos, ref["pos"])
    assert np.array_equal(vel, ref["vel"]) and np.array_equal(rho, ref["rhop"])


@need_ref
def test_reference_restarts_from_our_files(tmp_path):
    """-partbegin from a PART + Part_Head.ibi4 written here gives the reference's own
    restart, byte for byte."""
    src = tmp_path / "ours"
    src.mkdir()
    h, p = _restart_header(os.path.join(FIX, "Part_0001.bi4"))
    write_part(str(src / "Part_0001.bi4"), h, p)
    write_part_head(str(src / "Part_Head.ibi4"), h)
    case = tmp_path / "case"
    case.mkdir()
    for f in ("CaseDambreak.bi4", "CaseDambreak.xml"):
        shutil.copy(os.path.join(FIX, f), case / f)
    out = tmp_path / "rst"
    subprocess.check_call([os.path.join(REF, "DualSPHysics5.2CPU_ref"), str(case / "CaseDambreak"), str(out),
                           "-partbegin:1", str(src), "-nsteps:3", "-svsteps:1", "-nortimes:1", "-saveposdouble:1",
                           "-sv:binx", "-svres:0", "-ompthreads:2"], stdout=subprocess.DEVNULL)
    assert filecmp.cmp(str(out / "Part_0004.bi4"), os.path.join(FIX, "restart_Part_0004.bi4"), shallow=False)


@pytest.mark.gpu
def test_gpu_restart_from_reference_part(tmp_path):
    """The GPU solver continued from the reference's Part_0001 follows the reference's
    own restart (3 steps, the noise-floor tolerance of test_gpu_parity), and its state
    saves as a PART the reader round-trips."""
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    h, p = read_part(os.path.join(FIX, "Part_0001.bi4"))
    case = DamBreakCase(0.05).restart_from(h, p)
    s = SphGpuSingle(case, device=0)
    s.set_time(case.time0, case.symdtpre0)
    s.run(3)
    hr, pr = read_part(os.path.join(FIX, "restart_Part_0004.bi4"))
    got, ref = by_idp(s.particles()), by_idp(pr)
    assert np.array_equal(got["idp"], ref["idp"])
    assert abs(s.stats()["time"] - hr["timestep"]) <= 1e-9
    assert maxdiff(got, ref, "pos") <= 1e-7
    assert maxdiff(got, ref, "vel") <= 5e-5
    assert maxdiff(got, ref, "rhop") <= 1e-2
    f = str(tmp_path / "Part_0004.bi4")
    s.save_part(f, 4, head_path=str(tmp_path / "Part_Head.ibi4"))
    h2, p2 = read_part(f)
    assert h2["cpart"] == 4 and h2["npok"] == len(got["idp"])
    assert np.array_equal(by_idp(p2)["pos"], got["pos"])
