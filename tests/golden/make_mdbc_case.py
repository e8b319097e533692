"""Generate the mDBC case fixtures by running the REFERENCE solver (build container only:
needs the binaries of ``make -C oracle``).

tests/golden/bi4/mdbc/
  CaseDambreak.xml / .bi4 / _Normals.nbi4   case written by gencase_ref (dp 0.05, Verlet, DDT2,
                                            Boundary=2 SlipMode=1); the normals file through the
                                            reference's own JPartNormalData (JPartNormalData.cpp:178)
  Part_0020.bi4                             reference run -nsteps:20 -svsteps:1 -saveposdouble:1,
                                            its PART 20
Usage: python tests/golden/make_mdbc_case.py
"""
import os
import shutil
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref")
OUT = os.path.join(HERE, "bi4", "mdbc")


def main():
    os.makedirs(OUT, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="mdbc_")
    try:
        subprocess.check_call([os.path.join(REF, "gencase_ref"), "0.05", tmp, "1", "2", "1.5", "CaseDambreak", "2"],
                              stdout=subprocess.DEVNULL)
        for f in ("CaseDambreak.xml", "CaseDambreak.bi4", "CaseDambreak_Normals.nbi4"):
            shutil.copy(os.path.join(tmp, f), os.path.join(OUT, f))
        subprocess.check_call([os.path.join(REF, "DualSPHysics5.2CPU_ref"), os.path.join(tmp, "CaseDambreak"),
                               os.path.join(tmp, "out"), "-nsteps:20", "-svsteps:1", "-nortimes:1",
                               "-saveposdouble:1", "-sv:binx", "-svres:0", "-ompthreads:2"], stdout=subprocess.DEVNULL)
        shutil.copy(os.path.join(tmp, "out", "Part_0020.bi4"), os.path.join(OUT, "Part_0020.bi4"))
        print("written", sorted(os.listdir(OUT)))
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
