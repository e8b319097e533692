"""Generate the fixtures of the dt / viscosity options by running the REFERENCE solver (build
container only: needs the binaries of ``make -C oracle``).

tests/golden/bi4/dtopt_<variant>/
  Case*.xml / .bi4 [+ data files]   gencase_ref's dam break (or genflume_ref's flume) with the
                                    option's <parameter> added to <execution><parameters>:
                                    DtFixed (a constant dt), DtFixedFile (dt(t) in ms,
                                    JDsFixedDt), ViscoTime (Visco(t), JDsViscoInput),
                                    DtAllParticles (VelMax over every particle: the flume's
                                    fast flap, ~4 m/s at its tip, sets it)
  ref.npz                           the reference run (-nsteps:N -svsteps:1 -saveposdouble:1):
                                    PARTs at the kept steps (sorted by idp), every PART time,
                                    and noise_<k> = [dpos, dvel, drho] between the fast-math
                                    build and the strict build of the same sources
Usage: python tests/golden/make_dtopt_case.py [variant]
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
from make_golden import load_dump  # noqa: E402

# variant: (generator, dp, step 1 Verlet / 2 Symplectic, ddt, nsteps, kept steps, parameters, data files)
VARIANTS = {
    "verlet_ddt2_dtfixed": ("dambreak", 0.03, 1, 2, 100, (1, 10, 100), {"DtFixed": "2e-4"}, {}),
    "symplectic_ddt1_dtfixedfile": ("dambreak", 0.03, 2, 1, 60, (1, 20, 60), {"DtFixedFile": "dtfixed.csv"},
                                    {"dtfixed.csv": "# time(s);dt(ms)\n0;0.08\n0.006;0.22\n1;0.22\n"}),
    "verlet_ddt2_viscotime": ("dambreak", 0.03, 1, 2, 100, (1, 10, 100), {"ViscoTime": "visco.txt"},
                              {"visco.txt": "# time visco\n0 0.01\n0.004 0.6\n1 0.6\n"}),
    # rows out of time order: the reference walks them forward from the row of its last lookup
    # (JDsFixedDt::GetDt / JDsViscoInput::GetVisco keep Position), so past 6 ms the dt comes
    # from the (0.003 s, 1 s) interval, past 4 ms the Visco from the (0.002 s, 1 s) one
    "verlet_ddt2_dtfixedfile_unordered": ("dambreak", 0.03, 1, 2, 100, (1, 40, 100), {"DtFixedFile": "dtfixed.csv"},
                                          {"dtfixed.csv": "# time(s);dt(ms)\n0;0.08\n0.006;0.22\n0.003;0.15\n"
                                                          "1;0.3\n"}),
    "verlet_ddt2_viscotime_unordered": ("dambreak", 0.03, 1, 2, 100, (1, 50, 100), {"ViscoTime": "visco.txt"},
                                        {"visco.txt": "# time visco\n0 0.01\n0.004 0.6\n0.002 0.3\n1 0.1\n"}),
    # a fast wide flap (no wait, 8 Hz, 12 degrees): its tip, ~4 m/s, sets VelMax (10 VelMax > Cs0)
    "flume_verlet_ddt2_dtallparticles": ("flume", 0.03, 1, 2, 60, (1, 20, 60), {"DtAllParticles": "1"}, {}),
}


def make(name, gen, dp, step, ddt, nsteps, keep, params, files):
    out_dir = os.path.join(HERE, "bi4", "dtopt_" + name)
    os.makedirs(out_dir, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="dtopt_")
    try:
        case = "CaseDambreak" if gen == "dambreak" else "CaseFlume"
        if gen == "dambreak":
            cmd = [os.path.join(REF, "gencase_ref"), repr(dp), tmp, str(step), str(ddt), "1.5", case, "1", "3"]
        else:
            cmd = [os.path.join(REF, "genflume_ref"), repr(dp), tmp, str(step), str(ddt), "1.0", case, "1", "1.2",
                   "0.3", "0.4", "0.2", "0", "8", "12"]
        subprocess.check_call(cmd, stdout=subprocess.DEVNULL)
        fx = os.path.join(tmp, case + ".xml")
        txt = open(fx).read()
        assert txt.count("</parameters>") == 1
        add = "".join('<parameter key="%s" value="%s"/>\n' % kv for kv in params.items())
        open(fx, "w").write(txt.replace("</parameters>", add + "</parameters>"))
        for fn, body in files.items():
            open(os.path.join(tmp, fn), "w").write(body)
        for f in [case + ".xml", case + ".bi4"] + list(files):
            shutil.copy(os.path.join(tmp, f), os.path.join(out_dir, f))
        outs = {}
        for exe, tag in (("DualSPHysics5.2CPU_ref", "fast"), ("DualSPHysics5.2CPU_strict", "strict")):
            outs[tag] = os.path.join(tmp, "out_" + tag)
            subprocess.check_call([os.path.join(REF, exe), os.path.join(tmp, case), outs[tag], "-nsteps:%d" % nsteps,
                                   "-svsteps:1", "-nortimes:1", "-saveposdouble:1", "-sv:binx", "-svres:0",
                                   "-ompthreads:4"], stdout=subprocess.DEVNULL)
        arrays, times = {}, []
        fn = os.path.join(tmp, "p.bin")
        for part in range(nsteps + 1):
            subprocess.check_call([os.path.join(REF, "partdump_ref"), outs["fast"], str(part), fn],
                                  stdout=subprocess.DEVNULL)
            t, idp, pos, vel, rho = load_dump(fn)
            times.append(t)
            if part in keep:
                o = np.argsort(idp, kind="stable")
                idp, pos, vel, rho = idp[o], pos[o], vel[o], rho[o]
                arrays.update({"s%d_idp" % part: idp, "s%d_pos" % part: pos, "s%d_vel" % part: vel,
                               "s%d_rhop" % part: rho, "s%d_time" % part: np.float64(t)})
                subprocess.check_call([os.path.join(REF, "partdump_ref"), outs["strict"], str(part), fn],
                                      stdout=subprocess.DEVNULL)
                _, ids, poss, vels, rhos = load_dump(fn)
                os_ = np.argsort(ids, kind="stable")
                assert np.array_equal(idp, ids[os_]), "strict build excluded other particles"
                arrays["noise_%d" % part] = np.array([np.abs(pos - poss[os_]).max(), np.abs(vel - vels[os_]).max(),
                                                      np.abs(rho.astype(np.float64) - rhos[os_]).max()])
        arrays.update(times=np.array(times), meta=np.array([dp, step, ddt, nsteps], np.float64))
        np.savez_compressed(os.path.join(out_dir, "ref.npz"), **arrays)
        print(name, "ok", sorted(os.listdir(out_dir)), np.diff(times)[:3], np.diff(times)[-2:])
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    only = sys.argv[1] if len(sys.argv) > 1 else None
    for k, v in VARIANTS.items():
        if only is None or k == only:
            make(k, *v)
