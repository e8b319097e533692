"""Generate golden fixtures by running the REFERENCE DualSPHysics CPU solver.

Run in the build container only (needs /root/reference and the binaries built
by ``make -C oracle``: oracle/_ref/{DualSPHysics5.2CPU_ref,gencase_ref,partdump_ref}).
The reference runs the dam-break case written by gencase_ref with
``-nsteps:N -svsteps:1 -saveposdouble:1 -sv:binx`` and every selected
Part_XXXX.bi4 is converted by partdump_ref and stored (sorted by idp) as

    tests/golden/<name>.npz : idp, pos, vel, rhop, time  for each saved step
                              (keys s<step>_idp, s<step>_pos, ...)
                              plus dt trace ``dt`` (from the part times).

Viscosity / shifting variants (EXT_CASES) also store ext = [ViscoTreatment, Visco,
Shifting, ShiftCoef, ShiftTFS] and, with --noise, the reference's own rounding-noise floor
noise_<step> = [dpos, dvel, drho]: the largest differences between the fast-math build and
the same sources built without -ffast-math (``make -C oracle strict``).

Usage: python tests/golden/make_golden.py [--only NAME] [--noise]
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
    # 2-D mDBC (the sim2d branch of InteractionMdbcCorrectionT2, JSphCpu.cpp:1087-1110)
    "verlet_ddt2_mdbc_2d_dp0.02": (0.02, 1, 2, 100, (1, 10, 100), 2, (), 2),
    "symplectic_ddt1_mdbc_2d_dp0.02": (0.02, 2, 1, 60, (1, 20, 60), 2, (), 2),
    # Cubic spline kernel with its tensile correction (-cubic; FunSphKernel.h:38-175,
    # JSphCpu.cpp:713): the kernel of examples/main/01_DamBreak/CaseDambreak_Def.xml:68; the
    # npz carries kernel = 1
    "verlet_ddt2_cubic_dp0.02": (0.02, 1, 2, 100, (1, 10, 100), 1, ("-cubic",)),
    "symplectic_ddt1_cubic_mdbc_dp0.03": (0.03, 2, 1, 60, (1, 20, 60), 2, ("-cubic",)),
    "verlet_ddt2_cubic_2d_dp0.02": (0.02, 1, 2, 100, (1, 10, 100), 1, ("-cubic",), 2),
}

# Symmetry (<parameter Symmetry>, JSph.cpp:714): the half tank y >= 0 mirrored across y = 0
# (gencase_ref sym 1: no y = 0 wall, fluid from y = 0); the npz carries symmetry = 1.
# name: (dp, step, ddt, nsteps, kept steps, boundary)
SYM_CASES = {
    "verlet_ddt2_sym_dp0.02": (0.02, 1, 2, 100, (1, 10, 100), 1),
    "symplectic_ddt1_sym_mdbc_dp0.025": (0.025, 2, 1, 60, (1, 20, 60), 2),
}
# Symmetry with CellMode=half and with shifting (the reference refuses only 2-D, periodic y,
# floating bodies, Chrono and a viscosity other than the artificial one, JSph.cpp:1174-1179).
# name: (dp, step, ddt, nsteps, kept steps, boundary, extra args, (shifting, coef, tfs)); the
# npz adds ext = [1, 0.1, shifting, coef, tfs] as make_ext's
SYM_EXT_CASES = {
    "verlet_ddt2_sym_half_dp0.02": (0.02, 1, 2, 100, (1, 10, 100), 1, ("-cellmode:half",), (0, "-2", "0")),
    "symplectic_ddt2_sym_shift_full_tfs_dp0.025": (0.025, 2, 2, 60, (1, 20, 60), 1, (), (3, "-2", "2.75")),
    "verlet_ddt2_sym_shift_nobound_dp0.025": (0.025, 1, 2, 60, (1, 41, 60), 1, (), (1, "-2", "0")),
    "symplectic_ddt2_sym_shift_full_tfs_half_dp0.025": (0.025, 2, 2, 60, (1, 20, 60), 1, ("-cellmode:half",),
                                                        (3, "-2", "2.75")),
}


# Single-phase Laminar+SPS viscosity (ViscoTreatment 2; kinematic viscosity 1e-6 m2/s,
# JSphCpu.cpp:765-809, ComputeSpsTau :929-954) and shifting (JSphShifting, modes 1-3).
# name: (dp, step, ddt, nsteps, kept steps, (tvisco, visco, shifting, shiftcoef, shifttfs))
EXT_CASES = {
    "verlet_lamsps_ddt2_dp0.02": (0.02, 1, 2, 100, (1, 10, 100), (2, "1e-6", 0, "-2", "0")),
    "symplectic_lamsps_ddt1_dp0.025": (0.025, 2, 1, 60, (1, 20, 60), (2, "1e-6", 0, "-2", "0")),
    "verlet_shift_nobound_dp0.025": (0.025, 1, 2, 60, (1, 41, 60), (1, "0.1", 1, "-2", "0")),
    "symplectic_shift_full_tfs_dp0.025": (0.025, 2, 2, 60, (1, 20, 60), (1, "0.1", 3, "-2", "2.75")),
    "verlet_lamsps_shift_nofixed_dp0.03": (0.03, 1, 0, 45, (1, 41, 45), (2, "1e-6", 2, "-2", "1.5")),
}
# the same options with CellMode=half (-cellmode:half: cells of h, 5x5 rows; the npz
# carries cellmode = 2)
EXT_HALF_CASES = {
    "verlet_lamsps_ddt2_half_dp0.025": (0.025, 1, 2, 60, (1, 20, 60), (2, "1e-6", 0, "-2", "0")),
    "symplectic_shift_full_tfs_half_dp0.025": (0.025, 2, 2, 60, (1, 20, 60), (1, "0.1", 3, "-2", "2.75")),
    "verlet_lamsps_shift_nofixed_half_dp0.03": (0.03, 1, 0, 45, (1, 41, 45), (2, "1e-6", 2, "-2", "1.5")),
}
# The same physics from a STIRRED state (restart fixtures): a dam break at rest has no
# velocity gradient (no SPS stress) and no shifting displacement (|v| = 0) in its first
# steps, so these start from the generated case with every fluid particle given the smooth
# shear field of stir_velocity() plus a seeded random part, written as Part_0000 (the
# core's PART writer, byte-identical to the reference's, tests/test_bi4.py) as the PART
# of step 1 and run by the reference with -partbegin:1.  The npz adds s0_* (the stirred
# start) and rst = [time, SymplecticDtPre, map_posmin xyz, map_posmax xyz].
# (..., stir: "mild" or "shear" -- the strong short-wave shear under which the SPS eddy
# viscosity (Smagorinsky, ~SpsSmag |S| ~ 1e-4 m2/s) is far above the parity tolerance)
# Cubic spline kernel (-cubic, with its tensile correction) with Laminar+SPS and with
# shifting (JSphCpu.cpp:631-822 templated on tker for every tvisco / shift); the npz carries
# kernel = 1
EXT_CUBIC_CASES = {
    "verlet_lamsps_ddt2_cubic_dp0.02": (0.02, 1, 2, 100, (1, 10, 100), (2, "1e-6", 0, "-2", "0")),
    "symplectic_shift_full_tfs_cubic_dp0.025": (0.025, 2, 2, 60, (1, 20, 60), (1, "0.1", 3, "-2", "2.75")),
}
STIR_CUBIC_CASES = {
    "stir_verlet_lamsps_ddt2_cubic_dp0.025": (0.025, 1, 2, 40, (1, 10, 40), (2, "1e-6", 0, "-2", "0"), "shear"),
}
STIR_CASES = {
    "stir_verlet_lamsps_ddt2_dp0.025": (0.025, 1, 2, 40, (1, 10, 40), (2, "1e-6", 0, "-2", "0"), "shear"),
    "stir_symplectic_lamsps_ddt1_dp0.03": (0.03, 2, 1, 20, (1, 5, 20), (2, "1e-6", 0, "-2", "0"), "shear"),
    "stir_verlet_shift_full_tfs_dp0.025": (0.025, 1, 2, 40, (1, 10, 40), (1, "0.1", 3, "-2", "2.75"), "mild"),
    "stir_symplectic_lamsps_shift_nobound_dp0.03": (0.03, 2, 2, 20, (1, 5, 20), (2, "1e-6", 1, "-2", "0"), "shear"),
}


def stir_velocity(pos, idp, npb, kind="mild", seed=11):
    """Fluid particles (idp >= npb) get a shear field plus seeded uniform noise:
    mild:  u = 0.6 sin(2 pi z/0.3), v = 0.2 sin(2 pi y/0.67), w = 0.4 sin(2 pi x/0.4), +-0.15 m/s;
    shear: u = 1.5 sin(2 pi z/0.1), v = 0.5 sin(2 pi y/0.15), w = 1.0 sin(2 pi x/0.1), +-0.05 m/s."""
    rng = np.random.default_rng(seed)
    v = np.zeros((len(idp), 3), np.float32)
    fl = idp >= npb
    x, y, z = pos[fl, 0], pos[fl, 1], pos[fl, 2]
    if kind == "shear":
        a, l, noise = (1.5, 0.5, 1.0), (0.1, 0.15, 0.1), 0.05
    else:
        a, l, noise = (0.6, 0.2, 0.4), (0.3, 0.67, 0.4), 0.15
    v[fl, 0] = a[0] * np.sin(2 * np.pi * z / l[0])
    v[fl, 1] = a[1] * np.sin(2 * np.pi * y / l[1])
    v[fl, 2] = a[2] * np.sin(2 * np.pi * x / l[2])
    v[fl] += rng.uniform(-noise, noise, size=(int(fl.sum()), 3)).astype(np.float32)
    return v


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


def make(name, dp, step, ddt, nsteps, keep, boundary=1, extra=(), dim=3, noise=False, sym=False):
    tmp = tempfile.mkdtemp(prefix="golden_")
    try:
        gen = [os.path.join(REF, "gencase_ref"), repr(dp), tmp, str(step), str(ddt), "1.5", "CaseDambreak",
               str(boundary), str(dim)]
        if sym is True:  # artificial viscosity 0.1, no shifting, Wendland, Symmetry
            gen += ["1", "0.1", "0", "-2", "0", "2", "1"]
        elif sym:  # (shifting, coef, tfs): artificial viscosity 0.1, Wendland, Symmetry
            gen += ["1", "0.1", str(sym[0]), sym[1], sym[2], "2", "1"]
        subprocess.check_call(gen, stdout=subprocess.DEVNULL)
        out = os.path.join(tmp, "out")
        for exe, o in (("DualSPHysics5.2CPU_ref", out), ("DualSPHysics5.2CPU_strict", out + "_strict")):
            if o != out and not noise:
                continue
            subprocess.check_call(
                [os.path.join(REF, exe), os.path.join(tmp, "CaseDambreak"), o,
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
                if noise:  # the strict build's PART of the same step: the reference's noise floor
                    subprocess.check_call([os.path.join(REF, "partdump_ref"), out + "_strict", str(part), fn],
                                          stdout=subprocess.DEVNULL)
                    _, ids, poss, vels, rhos = load_dump(fn)
                    o, os_ = np.argsort(idp, kind="stable"), np.argsort(ids, kind="stable")
                    arrays["noise_%d" % part] = np.array([np.abs(pos[o] - poss[os_]).max(),
                                                          np.abs(vel[o] - vels[os_]).max(),
                                                          np.abs(rho[o] - rhos[os_]).max()])
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
        if "-cubic" in extra:
            arrays["kernel"] = np.int32(1)
        if sym:
            arrays["symmetry"] = np.int32(1)
        if sym and sym is not True:
            arrays["ext"] = np.array([1.0, 0.1, float(sym[0]), float(sym[1]), float(sym[2])], np.float64)
        np.savez_compressed(os.path.join(ROOT, "tests", "golden", name + ".npz"), **arrays)
        print(name, "ok", os.path.getsize(os.path.join(ROOT, "tests", "golden", name + ".npz")))
    finally:
        shutil.rmtree(tmp)


def run_ext(exe, dp, step, ddt, nsteps, ext, tmp, tag, extra=()):
    tv, visco, sh, coef, tfs = ext
    d = os.path.join(tmp, "case")
    os.makedirs(d, exist_ok=True)
    subprocess.check_call([os.path.join(REF, "gencase_ref"), repr(dp), d, str(step), str(ddt), "1.5", "CaseDambreak",
                           "1", "3", str(tv), visco, str(sh), coef, tfs], stdout=subprocess.DEVNULL)
    out = os.path.join(tmp, "out_" + tag)
    subprocess.check_call([exe, os.path.join(d, "CaseDambreak"), out, "-nsteps:%d" % nsteps, "-svsteps:1",
                           "-saveposdouble:1", "-sv:binx", "-svres:0"] + list(extra), stdout=subprocess.DEVNULL)
    return out


def make_stir(name, dp, step, ddt, nsteps, keep, ext, stir, noise, extra=()):
    sys.path.insert(0, ROOT)
    from dualsphysics_multilayer_amd.core import read_part, write_part

    tmp = tempfile.mkdtemp(prefix="golden_")
    try:
        tv, visco, sh, coef, tfs = ext
        d = os.path.join(tmp, "case")
        os.makedirs(d)
        subprocess.check_call([os.path.join(REF, "gencase_ref"), repr(dp), d, str(step), str(ddt), "1.5",
                               "CaseDambreak", "1", "3", str(tv), visco, str(sh), coef, tfs], stdout=subprocess.DEVNULL)
        # one step from rest: Part_0001 + Part_Head.ibi4 as the reference writes them; the
        # stirred state is that Part_0001 with new fluid velocities (-partbegin:0 is no
        # restart at all in JSph: PartBegin = 0 loads the case file)
        first = os.path.join(tmp, "first")
        subprocess.check_call([os.path.join(REF, "DualSPHysics5.2CPU_ref"), os.path.join(d, "CaseDambreak"), first,
                               "-nsteps:1", "-svsteps:1", "-saveposdouble:1", "-sv:binx", "-svres:0"] + list(extra),
                              stdout=subprocess.DEVNULL)
        h, p = read_part(os.path.join(first, "Part_0001.bi4"))
        npb = int(h["case_nfixed"])
        p["vel"] = stir_velocity(p["pos"], p["idp"], npb, stir)
        h.update(visco_type=int(tv), visco=float(visco), viscoboundfactor=1.0, gravity=[0.0, 0.0, -9.81], mkbound=10,
                 mkfluid=0)
        src = os.path.join(tmp, "src")
        os.makedirs(src)
        write_part(os.path.join(src, "Part_0001.bi4"), h, p)
        shutil.copy(os.path.join(first, "Part_Head.ibi4"), os.path.join(src, "Part_Head.ibi4"))

        def run(exe, tag):
            out = os.path.join(tmp, "out_" + tag)
            subprocess.check_call([exe, os.path.join(d, "CaseDambreak"), out, "-partbegin:1", src,
                                   "-nsteps:%d" % nsteps, "-svsteps:1", "-saveposdouble:1", "-sv:binx", "-svres:0"]
                                  + list(extra), stdout=subprocess.DEVNULL)
            return out

        out = run(os.path.join(REF, "DualSPHysics5.2CPU_ref"), "fast")
        outs = run(os.path.join(REF, "DualSPHysics5.2CPU_strict"), "strict") if noise else None
        o = np.argsort(p["idp"], kind="stable")
        arrays = {"s0_idp": p["idp"][o], "s0_pos": p["pos"][o], "s0_vel": p["vel"][o], "s0_rhop": p["rhop"][o],
                  "s0_time": np.float64(h["timestep"]),
                  "rst": np.array([h["timestep"], h["symplectic_dtpre"]] + list(h["map_posmin"]) +
                                  list(h["map_posmax"]), np.float64)}
        times = [h["timestep"]]
        fn = os.path.join(tmp, "p.bin")
        for k in range(1, nsteps + 1):  # step k after the restart = output part 1 + k
            subprocess.check_call([os.path.join(REF, "partdump_ref"), out, str(1 + k), fn], stdout=subprocess.DEVNULL)
            t, idp, pos, vel, rho = load_dump(fn)
            oo = np.argsort(idp, kind="stable")
            idp, pos, vel, rho = idp[oo], pos[oo], vel[oo], rho[oo]
            times.append(t)
            if k in keep:
                arrays.update({"s%d_idp" % k: idp, "s%d_pos" % k: pos, "s%d_vel" % k: vel,
                               "s%d_rhop" % k: rho, "s%d_time" % k: np.float64(t)})
                if outs:
                    subprocess.check_call([os.path.join(REF, "partdump_ref"), outs, str(1 + k), fn],
                                          stdout=subprocess.DEVNULL)
                    _, idps, poss, vels, rhos = load_dump(fn)
                    oo = np.argsort(idps, kind="stable")
                    assert np.array_equal(idp, idps[oo]), "strict build excluded other particles"
                    arrays["noise_%d" % k] = np.array([np.abs(pos - poss[oo]).max(), np.abs(vel - vels[oo]).max(),
                                                       np.abs(rho.astype(np.float64) - rhos[oo]).max()])
        arrays["times"] = np.array(times)
        arrays["dt"] = np.diff(np.array(times))
        arrays["meta"] = np.array([dp, step, ddt, nsteps], np.float64)
        arrays["ext"] = np.array([float(v) for v in ext], np.float64)
        if "-cubic" in extra:
            arrays["kernel"] = np.int32(1)
        np.savez_compressed(os.path.join(ROOT, "tests", "golden", name + ".npz"), **arrays)
        print(name, "ok", os.path.getsize(os.path.join(ROOT, "tests", "golden", name + ".npz")),
              {k: arrays[k] for k in arrays if k.startswith("noise")})
    finally:
        shutil.rmtree(tmp)


def make_ext(name, dp, step, ddt, nsteps, keep, ext, noise, extra=()):
    tmp = tempfile.mkdtemp(prefix="golden_")
    try:
        out = run_ext(os.path.join(REF, "DualSPHysics5.2CPU_ref"), dp, step, ddt, nsteps, ext, tmp, "fast", extra)
        outs = run_ext(os.path.join(REF, "DualSPHysics5.2CPU_strict"), dp, step, ddt, nsteps, ext, tmp,
                       "strict", extra) if noise else None
        arrays, times = {}, []
        fn = os.path.join(tmp, "p.bin")
        for part in range(nsteps + 1):
            subprocess.check_call([os.path.join(REF, "partdump_ref"), out, str(part), fn], stdout=subprocess.DEVNULL)
            t, idp, pos, vel, rho = load_dump(fn)
            o = np.argsort(idp, kind="stable")
            idp, pos, vel, rho = idp[o], pos[o], vel[o], rho[o]
            times.append(t)
            if part in keep:
                arrays.update({"s%d_idp" % part: idp, "s%d_pos" % part: pos, "s%d_vel" % part: vel,
                               "s%d_rhop" % part: rho, "s%d_time" % part: np.float64(t)})
                if outs:
                    subprocess.check_call([os.path.join(REF, "partdump_ref"), outs, str(part), fn],
                                          stdout=subprocess.DEVNULL)
                    _, idps, poss, vels, rhos = load_dump(fn)
                    o = np.argsort(idps, kind="stable")
                    assert np.array_equal(idp, idps[o]), "strict build excluded other particles"
                    arrays["noise_%d" % part] = np.array([np.abs(pos - poss[o]).max(), np.abs(vel - vels[o]).max(),
                                                          np.abs(rho.astype(np.float64) - rhos[o]).max()])
        arrays["times"] = np.array(times)
        arrays["dt"] = np.diff(np.array(times))
        arrays["meta"] = np.array([dp, step, ddt, nsteps], np.float64)
        arrays["ext"] = np.array([float(v) for v in ext], np.float64)
        if "-cellmode:half" in extra:
            arrays["cellmode"] = np.int32(2)
        if "-cubic" in extra:
            arrays["kernel"] = np.int32(1)
        np.savez_compressed(os.path.join(ROOT, "tests", "golden", name + ".npz"), **arrays)
        print(name, "ok", os.path.getsize(os.path.join(ROOT, "tests", "golden", name + ".npz")),
              {k: arrays[k] for k in arrays if k.startswith("noise")})
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
        make(name, *spec, **({"noise": True} if a.noise else {}))
    for name, spec in SYM_CASES.items():
        if a.only and a.only != name:
            continue
        make(name, *spec, noise=a.noise, sym=True)
    for name, spec in SYM_EXT_CASES.items():
        if a.only and a.only != name:
            continue
        make(name, *spec[:7], noise=a.noise, sym=spec[7])
    for name, spec in EXT_CASES.items():
        if a.only and a.only != name:
            continue
        make_ext(name, *spec, a.noise)
    for name, spec in EXT_HALF_CASES.items():
        if a.only and a.only != name:
            continue
        make_ext(name, *spec, a.noise, extra=("-cellmode:half",))
    for name, spec in STIR_CASES.items():
        if a.only and a.only != name:
            continue
        make_stir(name, *spec, a.noise)
    for name, spec in EXT_CUBIC_CASES.items():
        if a.only and a.only != name:
            continue
        make_ext(name, *spec, a.noise, extra=("-cubic",))
    for name, spec in STIR_CUBIC_CASES.items():
        if a.only and a.only != name:
            continue
        make_stir(name, *spec, a.noise, extra=("-cubic",))
