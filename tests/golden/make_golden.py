"""Generate golden fixtures by running the REFERENCE DualSPHysics CPU solver.

Run in the build container only (needs /root/reference and the binaries built
by ``make -C oracle``: oracle/_ref/{DualSPHysics5.2CPU_ref,gencase_ref,partdump_ref}).
The reference runs the dam-break case written by gencase_ref with
``-nsteps:N -svsteps:1 -saveposdouble:1 -sv:binx`` and every selected
Part_XXXX.bi4 is converted by partdump_ref and stored (sorted by idp) as

    tests/golden/<name>.npz : idp, pos, vel, rhop, time  for each saved step
                              (keys s<step>_idp, s<step>_pos, ...)
                              plus dt trace ``dt`` (from the part times).

Usage: python tests/golden/make_golden.py [--only NAME]
"""
import argparse
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = os.path.join(ROOT, "oracle", "_ref")

# name: (dp, step(1 Verlet/2 Symplectic), ddt, nsteps, steps kept[, boundary 1 DBC/2 mDBC[, extra options]])
CASES = {
    "verlet_ddt2_dp0.02": (0.02, 1, 2, 100, (1, 10, 100)),
    "symplectic_ddt1_dp0.025": (0.025, 2, 1, 100, (1, 10, 100)),
    "verlet_ddtnone_dp0.025": (0.025, 1, 0, 45, (1, 41, 45)),
    "symplectic_ddt3_dp0.03": (0.03, 2, 3, 20, (1, 20)),
    "verlet_ddt2_dp0.0127_dt": (0.0127, 1, 2, 100, ()),
    # mDBC (Boundary=2, SlipMode=1): normals from gencase_ref's <case>_Normals.nbi4
    "verlet_ddt2_mdbc_dp0.025": (0.025, 1, 2, 100, (1, 10, 100), 2),
    "symplectic_ddt1_mdbc_dp0.03": (0.03, 2, 1, 60, (1, 20, 60), 2),
    # CellMode=half (cells of h, 5x5 rows of 5 cells; JSph.cpp:1772-1788): meta[5] = 2
    "verlet_ddt2_half_dp0.025": (0.025, 1, 2, 60, (1, 20, 60), 1, ("-cellmode:half",)),
    # 2-D (Simulate2D): the CaseDambreakVal2D geometry (gencase_ref dim 2); meta[6] = 2
    "verlet_ddt2_2d_dp0.02": (0.02, 1, 2, 100, (1, 10, 100), 1, (), 2),
    "symplectic_ddt1_2d_dp0.02": (0.02, 2, 1, 60, (1, 20, 60), 1, (), 2),
}


def load_dump(fn):
    b = open(fn, "rb").read()
    n = int(np.frombuffer(b, np.uint32, 2)[1])
    t = float(np.frombuffer(b[8:16], np.float64)[0])
    o = 24
    idp = np.frombuffer(b, np.uint32, n, o); o += 4 * n
    pos = np.frombuffer(b, np.float64, 3 * n, o).reshape(n, 3); o += 24 * n
    vel = np.frombuffer(b, np.float32, 3 * n, o).reshape(n, 3); o += 12 * n
    rho = np.frombuffer(b, np.float32, n, o)
    return t, idp.copy(), pos.copy(), vel.copy(), rho.copy()


def make(name, dp, step, ddt, nsteps, keep, boundary=1, extra=(), dim=3):
    tmp = tempfile.mkdtemp(prefix="golden_")
    try:
        subprocess.check_call([os.path.join(REF, "gencase_ref"), repr(dp), tmp, str(step), str(ddt), "1.5",
                               "CaseDambreak", str(boundary), str(dim)], stdout=subprocess.DEVNULL)
        out = os.path.join(tmp, "out")
        subprocess.check_call(
            [os.path.join(REF, "DualSPHysics5.2CPU_ref"), os.path.join(tmp, "CaseDambreak"), out,
             "-nsteps:%d" % nsteps, "-svsteps:1", "-saveposdouble:1", "-sv:binx", "-svres:0"] + list(extra),
            stdout=subprocess.DEVNULL)
        arrays = {}
        times = []
        for part in range(nsteps + 1):
            fn = os.path.join(tmp, "p.bin")
            subprocess.check_call([os.path.join(REF, "partdump_ref"), out, str(part), fn], stdout=subprocess.DEVNULL)
            t, idp, pos, vel, rho = load_dump(fn)
            times.append(t)
            if part == 0:
                arrays["s0_sha_pos"] = np.frombuffer(__import__("hashlib").sha256(pos.tobytes()).digest(), np.uint8)
            if part in keep:
                arrays.update({"s%d_idp" % part: idp, "s%d_pos" % part: pos, "s%d_vel" % part: vel,
                               "s%d_rhop" % part: rho, "s%d_time" % part: np.float64(t)})
        arrays["times"] = np.array(times)
        arrays["dt"] = np.diff(np.array(times))
        m = [dp, step, ddt, nsteps]
        if boundary != 1 or extra or dim != 3:
            m.append(boundary)
        if "-cellmode:half" in extra or dim != 3:
            m.append(2 if "-cellmode:half" in extra else 1)
        if dim != 3:
            m.append(dim)
        arrays["meta"] = np.array(m, np.float64)
        np.savez_compressed(os.path.join(ROOT, "tests", "golden", name + ".npz"), **arrays)
        print(name, "ok", os.path.getsize(os.path.join(ROOT, "tests", "golden", name + ".npz")))
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only")
    a = ap.parse_args()
    for name, spec in CASES.items():
        if a.only and a.only != name:
            continue
        make(name, *spec)
