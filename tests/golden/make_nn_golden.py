"""Golden fixtures of the v5.0 NN multiphase solver (BASELINE cfg5).

Run in the build container only: needs the REFERENCE NN solver built from
src_mphase/DSPH_v5.0_NNewtonian/source by ``make -C oracle`` (oracle/_ref/
DualSPHysics5.0NN_CPU_ref) plus oracle/_ref/{gennn_ref,partdump_ref}.  Each case is the
3-D extruded wet dam break written by gennn_ref, run with ``-nsteps:N -svsteps:1
-saveposdouble:1 -sv:binx``; the kept PARTs are stored sorted by idp as

    tests/golden/nn_<name>.npz : s<step>_{idp,pos,vel,rhop,time}, times, dt, meta

meta = [dp, width, scale, shifttfs, velgrad, tvisco, ddt, shifting, csound, step, nsteps].

With ``--noise`` the same cases also run on the reference built WITHOUT -ffast-math
(``make -C oracle nnstrict``); the largest fast-math-vs-strict differences per kept step
are the reference's own rounding-noise floor (stored as noise_<step> = [dpos, dvel, drho]),
and the GPU tests hold the core to 10x that floor.

Usage: python tests/golden/make_nn_golden.py [--only NAME] [--noise]
"""
import argparse
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

# name: (dp, width, scale, shifttfs, velgrad, tvisco, ddt, shifting, csound, step, nsteps, kept steps)
CASES = {
    # the example's configuration (FDA, Laminar, DDT Fourtakas full, shifting Full), Symplectic
    "sym_lam_dp0.02": (0.02, 0.2, 0.5, 2.75, 1, 2, 3, 3, 0.0, 2, 60, (1, 10, 60)),
    # every phase with its own <csound>: DDT and phase CteB active; constitutive equation
    "sym_consteq_cs_dp0.025": (0.025, 0.2, 0.5, 2.75, 1, 3, 3, 3, 20.0, 2, 30, (1, 30)),
    # artificial viscosity with phase sound speeds, Molteni DDT, shifting NoBound, Verlet
    "ver_art_ddt1_cs_dp0.025": (0.025, 0.2, 0.5, 2.75, 1, 1, 1, 1, 20.0, 1, 45, (1, 41, 45)),
    # SPH velocity gradients (VelocityGradientType 2): gradients by SPH summation, then the
    # effective viscosity, then the Morris operator (Laminar) or the stress divergence (ConsEq)
    "sph_sym_lam_dp0.02": (0.02, 0.2, 0.5, 2.75, 2, 2, 3, 3, 0.0, 2, 60, (1, 10, 60)),
    "sph_sym_consteq_cs_dp0.025": (0.025, 0.2, 0.5, 2.75, 2, 3, 3, 3, 20.0, 2, 30, (1, 30)),
    "sph_ver_lam_ddt1_nobound_dp0.025": (0.025, 0.2, 0.5, 2.75, 2, 2, 1, 1, 0.0, 1, 45, (1, 41, 45)),
    # SPH gradients with artificial viscosity: the artificial term is the Morris pass's (bound p2
    # with dv = 2 v1), phase sound speeds
    "sph_ver_art_cs_dp0.025": (0.025, 0.2, 0.5, 2.75, 2, 1, 2, 0, 20.0, 1, 45, (1, 41, 45)),
    # CellMode=half (-cellmode:half: cells of h, 5x5 rows; the npz carries cellmode = 2)
    "sym_lam_half_dp0.02": (0.02, 0.2, 0.5, 2.75, 1, 2, 3, 3, 0.0, 2, 60, (1, 10, 60), ("-cellmode:half",)),
    "sph_sym_consteq_cs_half_dp0.025": (0.025, 0.2, 0.5, 2.75, 2, 3, 3, 3, 20.0, 2, 30, (1, 30),
                                        ("-cellmode:half",)),
    "ver_art_ddt1_cs_half_dp0.025": (0.025, 0.2, 0.5, 2.75, 1, 1, 1, 1, 20.0, 1, 45, (1, 41, 45),
                                     ("-cellmode:half",)),
    # a floating box (gennn_ref float 1: rhopbody 800 on the phase-0 layer; the npz carries
    # floating = 1): floating mass, the DDT and shifting rules of floating p1 / p2
    "ft_sym_lam_ddt3_dp0.025": (0.025, 0.4, 0.5, 2.75, 1, 2, 3, 3, 0.0, 2, 60, (1, 20, 60), (), 1),
    "ft_ver_art_ddt1_nobound_cs_dp0.025": (0.025, 0.4, 0.5, 2.75, 1, 1, 1, 1, 20.0, 1, 45, (1, 41, 45), (), 1),
    "ft_sph_sym_consteq_cs_dp0.025": (0.025, 0.4, 0.5, 2.75, 2, 3, 3, 3, 20.0, 2, 30, (1, 30), (), 1),
    # the floating body with CellMode=half (cells of h, 5x5 rows)
    "ft_sym_lam_ddt3_half_dp0.025": (0.025, 0.4, 0.5, 2.75, 1, 2, 3, 3, 0.0, 2, 60, (1, 20, 60), ("-cellmode:half",), 1),
    "ft_ver_art_ddt1_nobound_cs_half_dp0.025": (0.025, 0.4, 0.5, 2.75, 1, 1, 1, 1, 20.0, 1, 45, (1, 41, 45),
                                                ("-cellmode:half",), 1),
    # external forces on the floating body (FtSumExternalForces inside FtCalcForces of the v5.0
    # solver) and a ViscoTime table (Visco changes every step; the NN interactions take the
    # phases' viscosities, so it leaves the result unchanged): the npz carries xmledit
    "ft_sym_lam_ddt3_extforce_viscotime_dp0.025": (0.025, 0.4, 0.5, 2.75, 1, 2, 3, 3, 0.0, 2, 60, (1, 20, 60), (), 1,
                                                   "extforce_viscotime"),
}

# XML edits (anchor, text inserted before it) and data files written beside the case
XML_EDITS = {
    "extforce_viscotime": [
        ("</floating>", '<linearforce><force time="0" x="0.4" y="0" z="2"/><force time="0.02" x="-0.3" y="0.1" z="0.5"/>'
                        '</linearforce><angularforce><force time="0" x="0" y="0.002" z="0"/>'
                        '<force time="0.03" x="0.001" y="-0.002" z="0"/></angularforce>'),
        ("</parameters>", '<parameter key="ViscoTime" value="ViscoT.csv"/>\n'),
    ],
}
DATA_FILES = {"extforce_viscotime": {"ViscoT.csv": "# time;visco\n0;0.05\n0.01;0.2\n0.05;0.01\n"}}


def apply_edit(casedir, key):
    """The XML edit and data files of `key` on the case gennn_ref wrote into casedir."""
    fx = os.path.join(casedir, "CaseNN.xml")
    txt = open(fx).read()
    for anchor, text in XML_EDITS[key]:
        assert txt.count(anchor) == 1, anchor
        txt = txt.replace(anchor, text + anchor)
    open(fx, "w").write(txt)
    for fn, body in DATA_FILES.get(key, {}).items():
        open(os.path.join(casedir, fn), "w").write(body)


def run_case(exe, spec, tmp, nsteps):
    dp, width, scale, tfs, vg, tv, ddt, sh, cs, step = spec[:10]
    ft = str(spec[13]) if len(spec) > 13 else "0"
    subprocess.check_call([os.path.join(REF, "gennn_ref"), repr(dp), tmp, repr(width), repr(scale), "5",
                           "CaseNN", repr(tfs), str(vg), str(tv), str(ddt), str(sh), repr(cs), str(step), ft],
                          stdout=subprocess.DEVNULL)
    if len(spec) > 14 and spec[14]:
        apply_edit(tmp, spec[14])
    out = os.path.join(tmp, "out_" + os.path.basename(exe))
    extra = list(spec[12]) if len(spec) > 12 else []
    subprocess.check_call([exe, os.path.join(tmp, "CaseNN"), out, "-nsteps:%d" % nsteps, "-svsteps:1",
                           "-saveposdouble:1", "-sv:binx", "-svres:0"] + extra, stdout=subprocess.DEVNULL)
    return out


def dump(out, part, tmp):
    fn = os.path.join(tmp, "p.bin")
    subprocess.check_call([os.path.join(REF, "partdump_ref"), out, str(part), fn], stdout=subprocess.DEVNULL)
    t, idp, pos, vel, rho = load_dump(fn)
    o = np.argsort(idp, kind="stable")
    return t, idp[o], pos[o], vel[o], rho[o]


def make(name, spec, noise):
    nsteps, keep = spec[10], spec[11]
    tmp = tempfile.mkdtemp(prefix="nngolden_")
    try:
        out = run_case(os.path.join(REF, "DualSPHysics5.0NN_CPU_ref"), spec, tmp, nsteps)
        outs = run_case(os.path.join(REF, "DualSPHysics5.0NN_CPU_strict"), spec, tmp, nsteps) if noise else None
        arrays, times = {}, []
        for part in range(nsteps + 1):
            t, idp, pos, vel, rho = dump(out, part, tmp)
            times.append(t)
            if part in keep:
                arrays.update({"s%d_idp" % part: idp, "s%d_pos" % part: pos, "s%d_vel" % part: vel,
                               "s%d_rhop" % part: rho, "s%d_time" % part: np.float64(t)})
                if outs:
                    ts, idps, poss, vels, rhos = dump(outs, part, tmp)
                    assert np.array_equal(idp, idps), "strict build excluded other particles"
                    arrays["noise_%d" % part] = np.array([np.abs(pos - poss).max(), np.abs(vel - vels).max(),
                                                          np.abs(rho.astype(np.float64) - rhos).max()])
        arrays["times"] = np.array(times)
        arrays["dt"] = np.diff(np.array(times))
        arrays["meta"] = np.array(list(spec[:11]), np.float64)
        if len(spec) > 12 and "-cellmode:half" in spec[12]:
            arrays["cellmode"] = np.int32(2)
        if len(spec) > 13 and spec[13]:
            arrays["floating"] = np.int32(1)
        if len(spec) > 14 and spec[14]:
            arrays["xmledit"] = np.array(spec[14])
        fn = os.path.join(HERE, "nn_%s.npz" % name)
        np.savez_compressed(fn, **arrays)
        print(name, "ok", os.path.getsize(fn), {k: arrays[k] for k in arrays if k.startswith("noise")})
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only")
    ap.add_argument("--noise", action="store_true")
    a = ap.parse_args()
    for name, spec in CASES.items():
        if a.only and a.only != name:
            continue
        make(name, spec, a.noise)
