"""Run a case to TimeMax, saving PART files on the reference's output schedule
(the caller side of the hot path).

``CaseRun`` is the loop of ``JSphGpuSingle::Run`` (JSphGpuSingle.cpp:808-889) around
this core's steps:

  SaveData at the start (Part = PartIni, JSph::InitRun JSph.cpp:2210-2221), then per step
  TimeStep += dt; if TimeStep >= TimePartNext or the fluid fell below NpMinimum:
  SaveData, Part++, TimePartNext = next output time (``JDsOutputTime::GetNextTime``,
  JDsOutputTime.cpp:157-186; every step with -svsteps); stop at TimeMax or after
  NstepsBreak steps (-nsteps).

The core keeps TimeStep on the device, so the host cannot look at it after every step
without a round trip.  Steps are therefore issued in batches that provably cannot
cross the next output time: every dt the core computes is at most
``dt_cap = max(CFL*h/Cs0, DtMin)`` (``XmlCase.dt_cap``).  A Verlet step advances the time
by its own dt; a Symplectic step by the SymplecticDtPre of the step before
(JSphGpuSingle::ComputeStep_Sym; DtIni = h/Cs0 on the first step), known on the host at
the batch start.  So n steps advance by at most ``first + (n-1)*dt_cap`` and the largest
n keeping TimeStep < t_next is issued; near t_next the loop goes step by step.
The saved states and times are those of the reference's loop.  (Only the fluid-loss stop
``Np < NpMinimum``, which the reference checks every step, is seen at batch ends.)

A PART holds (JSph::SaveData / SavePartData, JSph.cpp:2581-2770): the particles in the
solver's cell order, TimeStep, Step (= steps done before this one), Nout (particles
excluded since the previous PART), the cell-domain limits of the last divide
(``JCellDivGpu::GetDomainLimits``, JCellDivGpu.cpp:391-400), SymplecticDtPre for
Symplectic; execution-dependent values (RunCode, Date, RunTime) as with -nortimes.
"""
from __future__ import annotations

import math
import os
import sys
import time

import numpy as np

from .core import SphGpuSingle, case_derive, write_part, write_part_head
from .xmlcase import CaseError, XmlCase


class OutputTime:
    """JDsOutputTime with one segment (TimeOut from the XML or -tout)."""

    def __init__(self, tout: float):
        if not tout > 0:
            raise CaseError("TimeOut must be positive.")
        self.tout = tout
        self._last_in = -1.0
        self._last_out = 0.0

    def next_time(self, t: float) -> float:
        if self._last_in >= 0 and t == self._last_in:
            return self._last_out
        self._last_in = t
        tb, tbout = 0.0, self.tout
        if t < tb:
            nxt = tb
        else:
            nt = int((t - tb) / tbout)
            nxt = tb + tbout * nt
            while nxt <= t:
                nxt = tb + tbout * nt
                nt += 1
        self._last_out = nxt
        return nxt


def cell_domain_limits(k: dict, pos: np.ndarray, npb: int) -> tuple[list, list]:
    """DomainMin/Max of a PART: the adaptive cell domain of JCellDivGpuSingle::CalcCellDomain
    (bound cells clipped to the fluid cells +- ScellDiv, JCellDivGpuSingle.cpp:47-99)
    mapped to positions by JCellDivGpu::GetDomainLimits."""
    dpm = np.asarray(k["dom_posmin"], np.float64)
    scell = float(k["scell"])
    ncell = np.asarray(k["dom_cells"], np.int64)
    sd = int(k["scelldiv"])
    cells = np.floor((pos - dpm) / scell).astype(np.int64)
    cells = np.clip(cells, 0, None)

    def limits(c):
        if not len(c):
            return ncell.copy(), np.zeros(3, np.int64)
        return c.min(axis=0), c.max(axis=0)

    bmin, bmax = limits(cells[:npb])
    fmin, fmax = limits(cells[npb:])
    cmin = np.maximum(np.minimum(bmin, fmin), np.where(fmin >= sd, fmin - sd, 0))
    cmax = np.minimum(np.maximum(bmax, fmax), fmax + sd)
    cmax = np.minimum(cmax, ncell - 1)
    if np.any(cmin > cmax):
        cmin = cmax = np.zeros(3, np.int64)
    lo, hi = cmin.copy(), cmax + 1
    for a in range(3):  # GetDomainLimits: an empty axis collapses to 0
        if cmin[a] > cmax[a]:
            lo[a] = hi[a] = 0
    return (dpm + scell * lo).tolist(), (dpm + scell * hi).tolist()


class _ExtraParts:
    """JDsExtraDataSave::Config + CheckSave (JDsExtraData.cpp:63-80): an interval n (every PART
    cpart > 0 with cpart % n == 0) or a JRangeFilter list such as "2,5-7"."""

    def __init__(self, spec: str):
        spec = str(spec).strip()
        self.every, self.allowed = 0, None
        if spec.isdigit():
            self.every = int(spec)
            return
        self.every, self.allowed = 1, set()
        for tok in spec.split(","):
            tok = tok.strip()
            a, _, b = tok.partition("-")
            if not a.isdigit() or (b and not b.isdigit()):
                raise CaseError(f"invalid SaveExtraParts value {spec!r}")
            self.allowed.update(range(int(a), int(b or a) + 1))

    def check(self, cpart: int) -> bool:
        return (cpart > 0 and self.every > 0 and cpart % self.every == 0
                and (self.allowed is None or cpart in self.allowed))


class CaseRun:
    """One case on one GPU from its initial (or restart) state to TimeMax."""

    def __init__(self, case: XmlCase, dirout: str, *, device: int = 0, nsteps_break: int = 0,
                 sv_all_steps: bool = False, sv_pos_double: bool = False, save: bool = True,
                 app_name: str = "dualsphysics_multilayer_amd", log=None, sv_extra_parts: str | None = None):
        self.case = case
        self.dirout = dirout
        self.nsteps_break = int(nsteps_break)
        self.sv_all_steps = bool(sv_all_steps)
        self.sv_pos_double = bool(sv_pos_double)
        self.save = save
        self.app_name = app_name
        self.log = log if log is not None else (lambda s: print(s, flush=True))
        self.k = case_derive(case.case_def())
        self.solver = SphGpuSingle(case, device=device)
        if case.time0 or case.symdtpre0:
            self.solver.set_time(case.time0, case.symdtpre0)
        # JSph::ConfigRunMode / LoadCaseConfig: NpMinimum=CaseNp-unsigned(PartsOutMax*CaseNfluid)
        self.npminimum = case.case_np - int(np.float32(case.partsoutmax) * np.float32(case.case_nfluid))
        self.output = OutputTime(case.timeout)
        self.parts: list[dict] = []
        self._nout_prev = 0
        self._ftparts: list[dict] = []
        # SaveExtraParts / -svextraparts (JSph.cpp:598,765; JDsExtraDataSave::Config): the mDBC
        # normals of every n-th PART (or of the listed PARTs), for a restart with mDBC
        sv = getattr(case, "sv_extra_parts", "") if sv_extra_parts is None else sv_extra_parts
        self._extra = _ExtraParts(sv) if (sv and case.tboundary == 2) else None
        if save:
            os.makedirs(dirout, exist_ok=True)

    # -- SaveData ------------------------------------------------------------------------------
    def _header(self, st: dict, cpart: int, step: int, nout: int) -> dict:
        c, cd = self.case, self.case.case_def()
        fb = [b for b in c.blocks if b["type"] == "fixed"]
        fl = [b for b in c.blocks if b["type"] == "fluid"]
        if not fl or not fb:
            raise CaseError("PART headers are written for cases with a fixed and a fluid block.")
        return dict(app_name=self.app_name, case_name=c.case_name, cpart=cpart, nout=nout, step=step,
                    timestep=float(st["time"]),
                    symplectic_dtpre=float(st["sym_dtpre"]) if c.step_algorithm == 2 else 0.0,
                    np_total=c.case_np, case_np=c.case_np, case_nfixed=c.case_nfixed, case_nfluid=c.case_nfluid,
                    case_nmoving=getattr(c, "case_nmoving", 0), case_nfloat=getattr(c, "case_nfloat", 0),
                    dp=c.dp, h=c.h, b=c.cteb, rhop0=c.rhop0, gamma=c.gamma, massbound=c.massbound,
                    massfluid=c.massfluid, map_posmin=list(cd["map_realposmin"]),
                    map_posmax=list(cd["map_realposmax"]), case_posmin=list(c.case_posmin),
                    case_posmax=list(c.case_posmax), pos_double=int(self.sv_pos_double), peri_mode=0,
                    visco_type=1, visco=float(np.float32(c.visco)),
                    viscoboundfactor=float(np.float32(c.viscoboundfactor)),
                    gravity=[float(np.float32(g)) for g in c.gravity], mkbound=fb[0]["mk"], mkfluid=fl[0]["mk"],
                    symmetry=int(cd.get("symmetry", 0)))  # JPartDataHead::ConfigSymmetry (JSph.cpp:2391)

    def _save(self, cpart: int, step: int) -> dict:
        st = self.solver.stats()
        nout = int(st["nout"]) - self._nout_prev
        self._nout_prev = int(st["nout"])
        info = dict(cpart=cpart, time=float(st["time"]), step=step, np=int(st["np"]), nout=nout)
        if self.save:
            p = self.solver.particles()
            hdr = self._header(st, cpart, step, nout)
            hdr["domain_min"], hdr["domain_max"] = cell_domain_limits(self.k, p["pos"], int(st["npb"]))
            write_part(os.path.join(self.dirout, "Part_%04u.bi4" % cpart), hdr,
                       {k: p[k] for k in ("idp", "pos", "vel", "rhop")})
            # Part_Head.ibi4 (restart header) lists one fixed and one fluid MK block; cases with
            # moving/floating blocks are not restartable by this core and get no Part_Head
            if not getattr(self.case, "has_bodies", False) and len(
                    [b for b in self.case.blocks if b["type"] == "fixed"]) == 1 and len(
                    [b for b in self.case.blocks if b["type"] == "fluid"]) == 1:
                write_part_head(os.path.join(self.dirout, "Part_Head.ibi4"), hdr)
            if self._extra is not None and self._extra.check(cpart):
                # PartExtra_%04u.bi4 (JSphGpuSingle::SaveExtraData, JSphGpuSingle.cpp:946-968)
                from .core import write_extra_normals

                nor, useft = self.solver.normals()
                nfl = int(getattr(self.case, "case_nfloat", 0))
                useft = useft and nfl > 0
                nsize = self.case.case_nbound if useft else self.case.case_nbound - nfl
                vnor = np.zeros((nsize, 3), np.float32)
                m = min(nsize, len(nor))
                vnor[:m] = nor[:m]
                write_extra_normals(os.path.join(self.dirout, "PartExtra_%04u.bi4" % cpart), self.app_name, cpart,
                                    step, float(st["time"]), self.case.case_nbound, nfl, vnor, useft)
            if getattr(self.case, "floatings", None):
                # PartFloat.fbi4: the body states of every saved PART (JSphCpuSingle SaveData ->
                # JPartFloatBi4Save::AddPartFloat/SavePartFloat)
                from .core import write_partfloat

                self._ftparts.append(dict(cpart=cpart, step=step, time=float(st["time"]),
                                          bodies=self.solver.floatings()))
                # rewritten whole into a temporary file and renamed over the previous one, so a
                # crash mid-write never truncates the records of earlier PARTs
                path = os.path.join(self.dirout, "PartFloat.fbi4")
                write_partfloat(path + ".tmp", self.case.floatings, self._ftparts,
                                mkboundfirst=self.case.mkboundfirst, app=self.app_name)
                os.replace(path + ".tmp", path)
        self.parts.append(info)
        self.log("Part_%04u  %12.6f  %12d  np=%u  out=%u" % (cpart, info["time"], step, info["np"], nout))
        return info

    # -- JSphGpuSingle::Run --------------------------------------------------------------------
    def run(self) -> list[dict]:
        case, sv = self.case, self.sv_all_steps
        cap = case.dt_cap()
        part = case.partbegin
        t0 = time.perf_counter()
        self._save(part, 0)
        part += 1
        st = self.solver.stats()
        t, nstep = float(st["time"]), 0
        tmax = case.timemax
        tnext = t if sv else self.output.next_time(t)
        while t < tmax:
            n = 1
            if not sv:
                # the next step advances by <= `first` (Symplectic: its SymplecticDtPre, which is
                # DtIni on the first step), every later one by <= cap
                first = float(st["sym_dtpre"]) * (1 + 1e-9) if case.step_algorithm == 2 else cap
                q = (min(tnext, tmax) - t - first) / cap
                n = max(1, math.ceil(q)) if q > 0 else 1
            if self.nsteps_break:
                n = min(n, self.nsteps_break - nstep)
            tprev = t
            self.solver.run(n)
            st = self.solver.stats()  # synchronises
            t = float(st["time"])
            if n > 1 and (t >= tnext or t >= tmax):
                raise RuntimeError(f"a batch of {n} steps crossed an output time ({tprev} -> {t}, dt_cap {cap})")
            if st["error_flags"]:
                raise RuntimeError(f"solver error flags {st['error_flags']:#x} at t={t}")
            nstep += n
            partoutstop = st["np"] < self.npminimum or not st["np"]
            if t >= tnext or partoutstop:
                if partoutstop:
                    self.log("**Particles OUT limit reached...")
                    tmax = t
                self._save(part, nstep - 1)
                part += 1
                tnext = t if sv else self.output.next_time(t)
            if self.nsteps_break and nstep >= self.nsteps_break:
                break
        self.elapsed = time.perf_counter() - t0
        self.nsteps = nstep
        self.log(f"Simulation finished: {nstep} steps, t={t:.6f} s, {self.elapsed:.2f} s wall")
        return self.parts

    def close(self) -> None:
        self.solver.close()


# ---- command line (the JSphCfgRun subset of this core) -------------------------------------
USAGE = """usage: python -m dualsphysics_multilayer_amd <case> [<dirout>] [options]
  <case>        case path without extension (<case>.xml + <case>.bi4)
  options (as DualSPHysics): -gpu[:id] -symplectic -verlet[:steps] -wendland -viscoart:v
  -viscoboundfactor:v -ddt:0..3 -ddtvalue:v -dbc -mdbc -mdbc_threshold:v -cellmode:full|half -cellfixed[:0|1]
  -saveposdouble[:0|1] -svextraparts:<n|list> -sv:binx|none -partbegin:n <dir> -rhopout:min:max -cfl:v -tmax:t
  -tout:t -domain_fixed:xmin:ymin:zmin:xmax:ymax:zmax -nsteps:n -svsteps[:0|1] -nortimes[:0|1]
  -dirout <dir> -name <case> -stable -svres -svtimers -ompthreads:n (accepted, no effect)"""


def _f32(s: str) -> float:
    return float(np.float32(float(s)))


def parse_args(argv: list[str]) -> dict:
    """JSphCfgRun::LoadArgv for the options this core runs; the rest raise CaseError."""
    o = dict(case=None, dirout=None, device=0, overrides={}, partbegin=0, partbegin_dir=None, nsteps=0,
             svsteps=False, nortimes=False, saveposdouble=False, save=True, domain_fixed=None, svextraparts=None)
    ov = o["overrides"]
    pos = []
    i = 0
    while i < len(argv):
        a = argv[i]
        if not a.startswith("-"):
            pos.append(a)
            i += 1
            continue
        w, _, rest = a[1:].partition(":")
        word, opts = w.upper(), (rest.split(":") if rest else [])
        full = rest

        def need_next():
            nonlocal i
            if i + 1 >= len(argv):
                raise CaseError(f"option {a} needs a value")
            i += 1
            return argv[i]

        if word == "GPU":
            o["device"] = int(full) if full else 0
        elif word == "CPU":
            raise CaseError("this core runs on the GPU (-cpu is the reference's CPU solver).")
        elif word == "DBC":
            ov["tboundary"], ov["slipmode"] = 1, 1
        elif word in ("STABLE", "SVRES", "SVTIMERS", "SVDOMAINVTK", "CREATEDIRS", "CSVSEP", "OMPTHREADS",
                      "WENDLAND"):
            pass  # the sort is always stable; logs / threads / defaults have no effect here
        elif word == "SAVEPOSDOUBLE":
            o["saveposdouble"] = (int(full) if full else 1) != 0
        elif word == "SVEXTRAPARTS":  # JSphCfgRun.cpp:287: PART interval or list of the extra data
            o["svextraparts"] = full
        elif word == "CELLMODE":
            v = full.upper()  # JSphCfgRun.cpp:295-299
            if v in ("HALF", "H"):
                ov["cellmode"] = 2
            elif v in ("", "FULL", "2H"):
                ov["cellmode"] = 1
            else:
                raise CaseError(f"invalid option {a}")
        elif word == "CELLFIXED":
            ov["celldomfixed"] = (int(full) if full else 1) != 0
        elif word == "MDBC":  # JSphCfgRun.cpp:306, JSph::LoadConfigCommands (JSph.cpp:766-790)
            ov["tboundary"], ov["slipmode"] = 2, 1
        elif word in ("MDBC_NOSLIP", "MDBC_FREESLIP"):
            raise CaseError("Only the slip mode velocity=0 is allowed with mDBC conditions.")
        elif word == "MDBC_THRESHOLD":
            v = _f32(full)
            if not 0 <= v:
                raise CaseError(f"invalid option {a}")
            ov["mdbc_threshold"] = v
        elif word == "MDBC_FAST":
            pass  # the correction is always accumulated and inverted in double (the CPU path)
        elif word in ("INITNORPLA", "INITNORPART", "SVNORMALS"):
            raise CaseError(f"-{w.lower()} is not supported by this core (normals come from <case>_Normals.nbi4).")
        elif word == "SYMPLECTIC":
            ov["step_algorithm"] = 2
        elif word == "VERLET":
            ov["step_algorithm"] = 1
            if full:
                ov["verlet_steps"] = int(full)
        elif word == "CUBIC":
            raise CaseError("Only the Wendland kernel runs on the GPU path.")
        elif word == "VISCOART":
            v = _f32(full)
            if v > 10:
                raise CaseError(f"invalid option {a}")
            ov["visco"], ov["tvisco"] = v, 1
        elif word == "VISCOLAMSPS":  # JSphCfgRun.cpp:329-333
            v = _f32(full)
            if v > 0.001:
                raise CaseError(f"invalid option {a}")
            ov["visco"], ov["tvisco"] = v, 2
        elif word == "VISCOBOUNDFACTOR":
            v = _f32(full)
            if v < 0:
                raise CaseError(f"invalid option {a}")
            ov["viscoboundfactor"] = v
        elif word == "DDT":
            v = int(full)
            if not 0 <= v <= 3:
                raise CaseError(f"invalid option {a}")
            ov["tdensity"] = v
        elif word == "DDTVALUE":
            v = _f32(full)
            if not 0 <= v <= 1:
                raise CaseError(f"invalid option {a}")
            ov["ddtvalue"] = v
        elif word == "SHIFTING":  # JSphCfgRun.cpp:355-362; JSph.cpp:825-835: ConfigBasic(mode) -> coef -2, TFS 0
            modes = {"NONE": 0, "NOBOUND": 1, "NOFIXED": 2, "FULL": 3}
            if full.upper() not in modes:
                raise CaseError(f"invalid option {a}")
            ov["shift_mode"], ov["shift_coef"], ov["shift_tfs"] = modes[full.upper()], -2.0, 0.0
        elif word == "SV":
            kinds = {s.strip().lower() for s in full.split(",") if s.strip()}
            bad = kinds - {"binx", "none", "info", "+binx", "-binx", "-csv", "-vtk", "-info", "+info"}
            if bad:
                raise CaseError(f"output formats {sorted(bad)} are not supported (PART .bi4 only).")
            o["save"] = any(k in ("binx", "+binx") for k in kinds)
        elif word == "NAME":
            o["case"] = need_next()
        elif word == "RUNNAME":
            need_next()
        elif word == "DIROUT":
            o["dirout"] = need_next()
        elif word == "DIRDATAOUT":
            raise CaseError("-dirdataout is not supported (PARTs go to the output directory).")
        elif word == "PARTBEGIN":
            o["partbegin"] = int(opts[0]) if opts else 0
            if len(opts) > 1 and opts[1] and int(opts[1]) != o["partbegin"]:
                raise CaseError("-partbegin:n:first with first != n is not supported.")
            o["partbegin_dir"] = need_next()
        elif word == "RHOPOUT":
            ov["rhopoutmin"], ov["rhopoutmax"] = _f32(opts[0]), _f32(opts[1])
        elif word == "CFL":
            v = float(full)
            if v <= 0:
                raise CaseError(f"invalid option {a}")
            ov["cflnumber"] = v
        elif word == "FTPAUSE":
            pass  # no floating bodies here
        elif word == "TMAX":
            ov["timemax"] = _f32(full)
        elif word == "TOUT":
            ov["timeout"] = _f32(full)
        elif word == "DOMAIN_FIXED":
            vals = [float(v) for v in opts]
            if len(vals) != 6:
                raise CaseError("-domain_fixed needs xmin:ymin:zmin:xmax:ymax:zmax")
            o["domain_fixed"] = vals
        elif word == "NSTEPS":
            o["nsteps"] = int(full)
            if o["nsteps"]:
                o["nortimes"] = True
        elif word == "SVSTEPS":
            o["svsteps"] = (int(full) if full else 1) != 0
            if o["svsteps"]:
                o["nortimes"] = True
        elif word == "NORTIMES":
            o["nortimes"] = (int(full) if full else 1) != 0
        elif word in ("H", "HELP", "?"):
            o["help"] = True
        else:
            raise CaseError(f"option {a} is not supported by this core.")
        i += 1
    if pos:
        o["case"] = o["case"] or pos[0]
    if len(pos) > 1:
        o["dirout"] = o["dirout"] or pos[1]
    return o


def load_from_args(o: dict) -> XmlCase:
    if not o["case"]:
        raise CaseError("Name of the case for execution was not indicated.")
    ov = dict(o["overrides"])
    if o.get("domain_fixed"):
        ov["domain_fixed"] = o["domain_fixed"]
    return XmlCase(o["case"], o["partbegin"], o["partbegin_dir"], **ov)


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    try:
        o = parse_args(argv)
        if o.get("help") or not o["case"]:
            print(USAGE)
            return 0 if o.get("help") else 1
        case = load_from_args(o)
        dirout = o["dirout"] or os.path.join(os.path.dirname(o["case"]) or ".", case.case_name + "_out")
        r = CaseRun(case, dirout, device=o["device"], nsteps_break=o["nsteps"], sv_all_steps=o["svsteps"],
                    sv_pos_double=o["saveposdouble"], save=o["save"], sv_extra_parts=o["svextraparts"])
        try:
            r.run()
        finally:
            r.close()
    except CaseError as e:
        print(f"*** Exception: {e}", file=sys.stderr)
        return 1
    return 0
