"""Generate the .bi4 fixtures by running the REFERENCE solver (build container only:
needs the binaries of ``make -C oracle``).

tests/golden/bi4/
  CaseDambreak.bi4 / CaseDambreak.xml  case written by gencase_ref (dp 0.05, Verlet, DDT2)
  Part_0001.bi4, Part_0004.bi4, Part_Head.ibi4
                                       reference run, -nsteps:4 -svsteps:1 -nortimes:1
                                       -saveposdouble:1 (files as the reference writes them)
  restart_Part_0004.bi4                reference run restarted from Part_0001 (-partbegin:1),
                                       its PART 4 (the golden of a restart)
  part1_ref_reader.npz                 Part_0001 as the reference's own reader returns it
                                       (partdump_ref, sorted by idp)
Usage: python tests/golden/make_bi4.py
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
OUT = os.path.join(HERE, "bi4")
sys.path.insert(0, HERE)
from make_golden import load_dump  # noqa: E402


def main():
    tmp = tempfile.mkdtemp(prefix="bi4_")
    try:
        subprocess.check_call([os.path.join(REF, "gencase_ref"), "0.05", tmp, "1", "2"], stdout=subprocess.DEVNULL)
        run = [os.path.join(REF, "DualSPHysics5.2CPU_ref"), os.path.join(tmp, "CaseDambreak")]
        opts = ["-nortimes:1", "-saveposdouble:1", "-sv:binx", "-svres:0", "-ompthreads:2"]
        subprocess.check_call(run + [os.path.join(tmp, "out"), "-nsteps:4", "-svsteps:1"] + opts,
                              stdout=subprocess.DEVNULL)
        subprocess.check_call(run + [os.path.join(tmp, "rst"), "-partbegin:1", os.path.join(tmp, "out"),
                                     "-nsteps:3", "-svsteps:1"] + opts, stdout=subprocess.DEVNULL)
        os.makedirs(OUT, exist_ok=True)
        for f in ("CaseDambreak.bi4", "CaseDambreak.xml"):
            shutil.copy(os.path.join(tmp, f), os.path.join(OUT, f))
        for f in ("Part_0001.bi4", "Part_0004.bi4", "Part_Head.ibi4"):
            shutil.copy(os.path.join(tmp, "out", f), os.path.join(OUT, f))
        shutil.copy(os.path.join(tmp, "rst", "Part_0004.bi4"), os.path.join(OUT, "restart_Part_0004.bi4"))
        dump = os.path.join(tmp, "p1.bin")
        subprocess.check_call([os.path.join(REF, "partdump_ref"), os.path.join(tmp, "out"), "1", dump],
                              stdout=subprocess.DEVNULL)
        t, idp, pos, vel, rho = load_dump(dump)
        np.savez(os.path.join(OUT, "part1_ref_reader.npz"), time=t, idp=idp, pos=pos, vel=vel, rhop=rho)
        print("written", sorted(os.listdir(OUT)))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
