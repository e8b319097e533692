"""Generate the restart fixtures of the wave flume (floating body, mDBC) by running the
REFERENCE solver (build container only: needs the binaries of ``make -C oracle``).

tests/golden/bi4/flumerst_<variant>/
  CaseFlume.xml / .bi4 [/ _Normals.nbi4]   the case (genflume_ref, as make_flume_case.py)
  Part_%04u.bi4 (PART k0)                  run A (-svsteps:1 -saveposdouble:1 [-svextraparts:1]):
  PartFloat.fbi4, [PartExtra_%04u.bi4]     the restart state at PART k0 — particles, the body
                                           states of PARTs 0..k0 (JPartFloatBi4), mDBC normals
  rst.npz                                  run B = the reference restarted from A's files at
                                           PART k0 (-partbegin:k0 <dirA>): its PARTs k0+1 ..
                                           k0+n (partdump_ref, sorted by idp), their times and
                                           body states (ftdump_ref); plus run A's own PART
                                           k0+n, whose distance to B's bounds how far a restart
                                           may drift from the uninterrupted run.
Usage: python tests/golden/make_flume_restart.py
"""
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref")
sys.path.insert(0, HERE)
from make_flume_case import load_ft  # noqa: E402
from make_golden import load_dump  # noqa: E402

FTNOR = ("1.2", "0.3", "0.4", "0.2", "0.004", "2", "3", "1")  # genflume_ref extras: floating normals
# variant: (dp, step, ddt, boundary, genflume extras, k0 restart PART, n steps after it)
VARIANTS = {
    "verlet_ddt2": (0.025, 1, 2, 1, (), 10, 10),
    "symplectic_ddt1_mdbc_ftnor": (0.025, 2, 1, 2, FTNOR, 8, 8),
}


def dump_parts(out, parts, tmp):
    arrays, times = {}, []
    for part in parts:
        fn = os.path.join(tmp, "p.bin")
        subprocess.check_call([os.path.join(REF, "partdump_ref"), out, str(part), fn], stdout=subprocess.DEVNULL)
        t, idp, pos, vel, rho = load_dump(fn)
        times.append(t)
        arrays.update({"s%d_idp" % part: idp, "s%d_pos" % part: pos, "s%d_vel" % part: vel,
                       "s%d_rhop" % part: rho, "s%d_time" % part: np.float64(t)})
    return arrays, times


def make(name, dp, step, ddt, boundary, extra, k0, n):
    out_dir = os.path.join(HERE, "bi4", "flumerst_" + name)
    if os.path.isdir(out_dir):
        shutil.rmtree(out_dir)
    os.makedirs(out_dir)
    tmp = tempfile.mkdtemp(prefix="flumerst_")
    exe = os.path.join(REF, "DualSPHysics5.2CPU_ref")
    common = ["-svsteps:1", "-nortimes:1", "-saveposdouble:1", "-sv:binx", "-svres:0", "-ompthreads:4"]
    try:
        subprocess.check_call([os.path.join(REF, "genflume_ref"), repr(dp), tmp, str(step), str(ddt), "1.0",
                               "CaseFlume", str(boundary)] + list(extra), stdout=subprocess.DEVNULL)
        files = ["CaseFlume.xml", "CaseFlume.bi4"] + (["CaseFlume_Normals.nbi4"] if boundary == 2 else [])
        for f in files:
            shutil.copy(os.path.join(tmp, f), os.path.join(out_dir, f))
        case = os.path.join(tmp, "CaseFlume")
        a = os.path.join(tmp, "a")
        subprocess.check_call([exe, case, a, "-nsteps:%d" % (k0 + n)] + common
                              + (["-svextraparts:1"] if boundary == 2 else []), stdout=subprocess.DEVNULL)
        # the restart state at PART k0
        rst = ["Part_%04u.bi4" % k0, "PartFloat.fbi4"] + (["PartExtra_%04u.bi4" % k0] if boundary == 2 else [])
        for f in rst:
            shutil.copy(os.path.join(a, f), os.path.join(out_dir, f))
        b = os.path.join(tmp, "b")
        subprocess.check_call([exe, case, b, "-partbegin:%d" % k0, a, "-nsteps:%d" % n]
                              + common, stdout=subprocess.DEVNULL)
        arrays, times = dump_parts(b, range(k0 + 1, k0 + n + 1), tmp)
        subprocess.check_call([os.path.join(REF, "ftdump_ref"), b, os.path.join(tmp, "ft.bin")],
                              stdout=subprocess.DEVNULL)
        ft, fc, fv, fw = load_ft(os.path.join(tmp, "ft.bin"))
        aa, _ = dump_parts(a, [k0 + n], tmp)
        arrays.update({"a_" + k: v for k, v in aa.items()})
        arrays.update(times=np.array(times), ft_time=ft, ft_center=fc, ft_fvel=fv, ft_fomega=fw,
                      meta=np.array([dp, step, ddt, boundary, k0, n], np.float64))
        np.savez_compressed(os.path.join(out_dir, "rst.npz"), **arrays)
        print(name, "ok", sorted(os.listdir(out_dir)), "ft parts", len(ft))
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    only = sys.argv[1] if len(sys.argv) > 1 else None
    for k, v in VARIANTS.items():
        if only is None or k == only:
            make(k, *v)
