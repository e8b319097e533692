"""Developed-flow trace of the REFERENCE CPU solver on the 3-D dam break (the cfg2 case's
geometry and physics — Verlet, DDT2 0.1, artificial viscosity 0.1 — at dp 0.015, 36,936
particles), for tests/test_developed.py.

Runs DualSPHysics5.2CPU_ref to t = 1.0 s (the surge crosses the tank, hits the far wall at
~0.45 s, runs up, falls back and rolls back over the tank: the flow the bench's
`--developed-presteps` times) with the case's TimeOut (0.01 s) and stores, per PART, bulk
statistics of the fluid (`stats` below, shared with the test): the surge front x, the fluid's
centre of mass (x, z), its kinetic energy per unit mass and the number of fluid particles.
Run in the build container only (needs /root/reference and make -C oracle).

Usage: python tests/golden/make_3d_developed.py
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
from golden.make_golden import REF, load_dump  # noqa: E402

DP, STEP, DDT, TMAX = 0.015, 1, 2, 1.0
NAME = "developed_3d_verlet_ddt2_dp0.015"


def stats(idp, pos, vel, npb):
    """Per state: front x (all but 0.2 % of the fluid behind it), centre of mass x and z,
    kinetic energy per unit mass 0.5 <|v|^2>, fluid particles."""
    f = idp >= npb
    x = np.sort(pos[f, 0])
    v2 = (vel[f].astype(np.float64) ** 2).sum(axis=1)
    return np.array([x[-max(1, x.size // 500)], pos[f, 0].mean(), pos[f, 2].mean(), 0.5 * v2.mean(), f.sum()])


def run():
    tmp = tempfile.mkdtemp(prefix="dev3d_")
    try:
        subprocess.check_call([os.path.join(REF, "gencase_ref"), repr(DP), tmp, str(STEP), str(DDT), repr(TMAX),
                               "C3", "1", "3"], stdout=subprocess.DEVNULL)
        out = os.path.join(tmp, "out")
        subprocess.check_call([os.path.join(REF, "DualSPHysics5.2CPU_ref"), os.path.join(tmp, "C3"), out,
                               "-saveposdouble:1", "-sv:binx", "-svres:0", "-ompthreads:8"], stdout=subprocess.DEVNULL)
        times, rows = [], []
        part = 0
        while os.path.exists(os.path.join(out, "Part_%04d.bi4" % part)):
            fn = os.path.join(tmp, "p.bin")
            subprocess.check_call([os.path.join(REF, "partdump_ref"), out, str(part), fn], stdout=subprocess.DEVNULL)
            t, idp, pos, vel, _ = load_dump(fn)
            times.append(t)
            rows.append((idp, pos, vel))
            part += 1
        return np.array(times), rows
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    from dualsphysics_multilayer_amd.case import DamBreakCase

    npb = DamBreakCase(DP).npb
    times, parts = run()
    st = np.array([stats(i, p, v, npb) for i, p, v in parts])
    fn = os.path.join(HERE, NAME + ".npz")
    np.savez_compressed(fn, times=times, stats=st, meta=np.array([DP, STEP, DDT, TMAX], np.float64))
    print(NAME, len(times), "parts; front / com x / ke every 0.1 s:")
    print(np.round(st[::10, :4], 4))
