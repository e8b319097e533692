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
  sched_<tag>.json, sched_<tag>_last.bi4
                                       runs on the output schedule (-tmax / -tout): every PART's
                                       header values, and the last PART; tags: verlet (DDT2),
                                       sym_ddt1 (-symplectic -ddt:1), restart (verlet restarted
                                       from its Part_0002); sched_verlet_Part_0002.bi4 (the
                                       restart's input)
  domains.json                         map limits the reference derives for <simulationdomain>,
                                       legacy IncZ / DomainFixed* and -domain_fixed variants
                                       (variant_xml() writes each case XML)
Usage: python tests/golden/make_bi4.py
"""
import os
import json
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


SCHED_KEYS = ("cpart", "timestep", "step", "npok", "nout", "domain_min", "domain_max", "symplectic_dtpre")

# (name, posmin xyz, posmax xyz, extra <parameter>s, command-line options)
DOMAIN_VARIANTS = [
    ("base", ["default"] * 3, ["default", "default", "default + 50%"], {}, []),
    ("mixed", ["default - 0.1", "default-10%", "-0.05"], ["default + 20%", "2", "default+0.3"], {}, []),
    ("incz", ["default"] * 3, ["default"] * 3, {"IncZ": "0.7"}, []),
    ("fixedxmax", ["default"] * 3, ["default"] * 3, {"DomainFixedXmax": "2.5", "DomainFixedZmin": "-0.2"}, []),
    ("cli_fixed", ["default"] * 3, ["default", "default", "default + 50%"], {},
     ["-domain_fixed:-0.1:-0.1:-0.1:2:1:1"]),
]


def variant_xml(xml: str, posmin, posmax, params) -> str:
    """The generated case XML with another <simulationdomain> and extra parameters."""
    i, j = xml.index("<simulationdomain>"), xml.index("</simulationdomain>") + len("</simulationdomain>")
    dom = ('<simulationdomain><posmin x="%s" y="%s" z="%s"/><posmax x="%s" y="%s" z="%s"/></simulationdomain>'
           % (*posmin, *posmax))
    extra = "".join('<parameter key="%s" value="%s"/>\n' % kv for kv in params.items())
    return xml[:i] + extra + dom + xml[j:]


def read_header(path, keys=SCHED_KEYS):
    """PART values the tests compare (the container reader of the core library)."""
    sys.path.insert(0, ROOT)
    from dualsphysics_multilayer_amd.core import read_part

    h, p = read_part(path)
    return {k: h[k] for k in keys}


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
        sched = ["-tmax:0.01", "-tout:0.002", "-saveposdouble:1", "-sv:binx", "-svres:0", "-ompthreads:2",
                 "-nortimes:1"]
        for tag, extra, src in (("verlet", [], None), ("sym_ddt1", ["-symplectic", "-ddt:1"], None),
                                ("restart", ["-partbegin:2", os.path.join(tmp, "s_verlet")], "verlet")):
            d = os.path.join(tmp, "s_" + tag)
            subprocess.check_call(run + [d] + sched + extra, stdout=subprocess.DEVNULL)
            parts = sorted(f for f in os.listdir(d) if f.startswith("Part_") and f.endswith(".bi4"))
            summ = []
            for f in parts:
                summ.append(read_header(os.path.join(d, f)))
            with open(os.path.join(OUT, f"sched_{tag}.json"), "w") as fh:
                json.dump(summ, fh, indent=1)
            shutil.copy(os.path.join(d, parts[-1]), os.path.join(OUT, f"sched_{tag}_last.bi4"))
            if tag == "verlet":
                shutil.copy(os.path.join(d, "Part_0002.bi4"), os.path.join(OUT, "sched_verlet_Part_0002.bi4"))
        doms = []
        for name, posmin, posmax, params, cli in DOMAIN_VARIANTS:
            vd = os.path.join(tmp, "dom_" + name)
            os.makedirs(vd)
            shutil.copy(os.path.join(tmp, "CaseDambreak.bi4"), os.path.join(vd, "CaseDambreak.bi4"))
            with open(os.path.join(tmp, "CaseDambreak.xml")) as fh:
                xml = fh.read()
            with open(os.path.join(vd, "CaseDambreak.xml"), "w") as fh:
                fh.write(variant_xml(xml, posmin, posmax, params))
            subprocess.check_call([run[0], os.path.join(vd, "CaseDambreak"), os.path.join(vd, "out"), "-nsteps:1",
                                   "-sv:binx", "-svres:0", "-ompthreads:2"] + cli, stdout=subprocess.DEVNULL)
            h = read_header(os.path.join(vd, "out", "Part_0000.bi4"), ("map_posmin", "map_posmax"))
            doms.append(dict(name=name, posmin=posmin, posmax=posmax, params=params, cli=cli, **h))
        with open(os.path.join(OUT, "domains.json"), "w") as fh:
            json.dump(doms, fh, indent=1)
        print("written", sorted(os.listdir(OUT)))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
