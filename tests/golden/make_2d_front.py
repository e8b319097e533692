"""Surge-front trace of the REFERENCE CPU solver on the 2-D dam break (CaseDambreakVal2D
geometry, oracle/tools/gencase_ref dim 2), for tests/test_2d.py.

Runs DualSPHysics5.2CPU_ref to t = 0.76 s with the case's TimeOut (0.01 s), reads every
PART with partdump_ref and stores, per PART, its time and the dam tip x (front statistic
`tip_x` below, shared with the test) in tests/golden/front_2d_<name>.npz.
Run in the build container only (needs /root/reference and make -C oracle).

Usage: python tests/golden/make_2d_front.py
"""
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from golden.make_golden import REF, ROOT, load_dump  # noqa: E402

# name: (dp, step algorithm, ddt)
CASES = {"verlet_ddt2_dp0.02": (0.02, 1, 2)}
TMAX = 0.76


def tip_x(idp, pos, npb):
    """Dam tip: the x below which all but 0.2% of the fluid particles lie (drops off the
    front do not count)."""
    x = np.sort(pos[idp >= npb, 0])
    return float(x[-max(1, x.size // 500)])


def make(name, dp, step, ddt):
    tmp = tempfile.mkdtemp(prefix="front_")
    try:
        subprocess.check_call([os.path.join(REF, "gencase_ref"), repr(dp), tmp, str(step), str(ddt), repr(TMAX),
                               "C2", "1", "2"], stdout=subprocess.DEVNULL)
        out = os.path.join(tmp, "out")
        subprocess.check_call([os.path.join(REF, "DualSPHysics5.2CPU_ref"), os.path.join(tmp, "C2"), out,
                               "-saveposdouble:1", "-sv:binx", "-svres:0"], stdout=subprocess.DEVNULL)
        times, tips = [], []
        part = 0
        while os.path.exists(os.path.join(out, "Part_%04d.bi4" % part)):
            fn = os.path.join(tmp, "p.bin")
            subprocess.check_call([os.path.join(REF, "partdump_ref"), out, str(part), fn], stdout=subprocess.DEVNULL)
            t, idp, pos, _, _ = load_dump(fn)
            times.append(t)
            tips.append((idp, pos))
            part += 1
        return np.array(times), tips
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    from dualsphysics_multilayer_amd.case import DamBreak2DCase

    for name, (dp, step, ddt) in CASES.items():
        npb = DamBreak2DCase(dp).npb
        times, parts = make(name, dp, step, ddt)
        tips = np.array([tip_x(i, p, npb) for i, p in parts])
        fn = os.path.join(HERE, "front_2d_%s.npz" % name)
        np.savez_compressed(fn, times=times, tip=tips, meta=np.array([dp, step, ddt], np.float64))
        print(name, len(times), "parts", "tips", np.round(tips[::10], 3))
