"""A DualSPHysics case as the reference solver loads it: ``<case>.xml`` + ``<case>.bi4``
(SURVEY.md §8(f) row 2).

Mirrors what ``JSph`` reads before the first step, restricted to what the hot path of
this core runs (fixed and moving DBC/mDBC boundaries, RigidAlgorithm=1 floating bodies, fluid,
Wendland, artificial viscosity, DDT 0-3,
Verlet / Symplectic, no periodicity); anything else raises ``CaseError`` the way the
reference refuses an invalid configuration, never silently ignored:

* constants  — ``JCaseCtes::ReadXmlRun`` (JCaseCtes.cpp:201-215) via
  ``JSph::LoadConfigCtes`` (JSph.cpp:567-583);
* parameters — ``JCaseEParms::ReadXml`` (JCaseEParms.cpp:351-375) and the keys and
  defaults of ``JSph::LoadConfigParameters`` (JSph.cpp:588-757), including the
  ``<simulationdomain>`` grammar of ``JCaseEParms::CheckPosValue``
  (JCaseEParms.cpp:283-320) and the legacy IncZ / DomainFixed* keys;
* command-line overrides — the subset of ``JSph::LoadConfigCommands``
  (JSph.cpp:762-870) this core supports (``overrides`` below);
* particle blocks — ``JCaseParts`` (``<particles>``) and the block codes of
  ``JSphMk::Config`` (JSphMk.cpp:86-123);
* particles and map limits — ``JSph::LoadCaseParticles`` (JSph.cpp:2036-2062):
  ``JPartsLoad4::LoadParticles`` (JPartsLoad4.cpp:151-252) from the case file or, for a
  restart (``partbegin``), from ``Part_%04u.bi4``; the map is the file's MapPosMin/Max
  when stored, else ``CalculeLimits`` (JPartsLoad4.cpp:339-347) + ``ResizeMapLimits``
  (JSph.cpp:1354-1387).

The solver holds boundary particles before fluid ones (``SphCaseDef.npb`` leading
entries).  Particles are therefore stably partitioned bound-first; the divide's cell
sort is stable and bound/fluid never share a box, so the sorted order the reference
builds from the file order is unchanged.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET

import numpy as np

from .case import BORDER_MAP, CELLMODE_FULL, CODE_TYPE_FIXED, CODE_TYPE_FLUID

DBL_MAX = float(np.finfo(np.float64).max)
CODE_TYPE_MOVING, CODE_TYPE_FLOATING = 0x800, 0x1000  # 16-bit typecode, DualSphDef.h:200-205


def _read_datafile(path: str, what: str, nvalues: int = 1, special: bool = False) -> np.ndarray:
    """Rows of (time, value...) of a JReadDatafile table (JDsFixedDt / JDsViscoInput /
    JLinearValue::LoadFile, JLinearValue.cpp:427-452): '#' lines are remarks, the separator is
    the most frequent of tab/space, ';' and ',', values are read as atof reads them ("none" is
    DBL_MAX where the table allows special values); at least two rows."""
    if not os.path.isfile(path):
        raise CaseError(f"{what}: file not found {path}")
    lines = [ln.strip() for ln in open(path).read().replace("\r", "").split("\n")]
    lines = [ln for ln in lines if ln and not ln.startswith("#")]
    head = "".join(lines[:20])
    ws, sc, cm = head.count(" ") + head.count("\t"), head.count(";"), head.count(",")
    sep = None if ws >= sc and ws >= cm else (";" if sc >= cm else ",")

    def atof(v: str) -> float:
        import re

        m = re.match(r"\s*[-+]?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?", v)
        return float(m.group(0)) if m else 0.0

    rows = []
    for ln in lines:
        f = ln.split(sep) if sep else ln.split()
        if len(f) < 1 + nvalues:
            raise CaseError(f"{what}: value {len(f) + 1} does not exist in line '{ln}' of {path}")
        rows.append((atof(f[0]),) + tuple(DBL_MAX if special and v.strip().lower() == "none" else atof(v)
                                         for v in f[1:1 + nvalues]))
    if len(rows) < 2:
        raise CaseError(f"{what}: Cannot be less than two values. ({path})")
    return np.array(rows, np.float64)


def _read_datafile_cols(path: str, what: str, ncols: int) -> np.ndarray:
    """Every row's first ncols values of a JReadDatafile table (separators and remarks as
    _read_datafile; JMotionDataFile::LoadFilePos / LoadFileAng, JMotionMov.cpp:252-300)."""
    if not os.path.isfile(path):
        raise CaseError(f"{what}: file not found {path}")
    lines = [ln.strip() for ln in open(path).read().replace("\r", "").split("\n")]
    lines = [ln for ln in lines if ln and not ln.startswith("#")]
    head = "".join(lines[:20])
    ws, sc, cm = head.count(" ") + head.count("\t"), head.count(";"), head.count(",")
    sep = None if ws >= sc and ws >= cm else (";" if sc >= cm else ",")
    import re

    def atof(v: str) -> float:
        m = re.match(r"\s*[-+]?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?", v)
        return float(m.group(0)) if m else 0.0

    rows = []
    for ln in lines:
        f = ln.split(sep) if sep else ln.split()
        if len(f) < ncols:
            raise CaseError(f"{what}: value {len(f) + 1} does not exist in line '{ln}' of {path}")
        rows.append(tuple(atof(v) for v in f[:ncols]))
    return np.array(rows, np.float64).reshape(-1, ncols)


class CaseError(ValueError):
    """An invalid or unsupported case configuration (the reference's JException)."""


# ---- XML helpers (JXml semantics) --------------------------------------------------------
def _node(root, path: str, optional: bool = False):
    n = root
    for part in path.split("."):
        n = n.find(part) if n is not None else None
    if n is None and not optional:
        raise CaseError(f"The item is not found '{path}'.")
    return n


def _attr_double(ele, name: str, what: str) -> float:
    v = ele.get(name)
    if v is None:
        raise CaseError(f"The attribute '{name}' of '{what}' is missing.")
    try:
        return float(v)
    except ValueError:
        raise CaseError(f"The attribute '{name}' of '{what}' is not a number: {v!r}") from None


def _elem_double(node, name: str, optional: bool = False, default: float = 0.0) -> float:
    e = node.find(name)
    if e is None:
        if optional:
            return default
        raise CaseError(f"The item is not found '{name}'.")
    return _attr_double(e, "value", name)


def _elem_bool(node, name: str) -> bool:
    e = node.find(name)
    if e is None:
        raise CaseError(f"The item is not found '{name}'.")
    v = (e.get("value") or "").strip().lower()
    if v in ("true", "1"):
        return True
    if v in ("false", "0"):
        return False
    raise CaseError(f"The value of '{name}' is not a valid boolean: {v!r}")


# ---- <simulationdomain> (JCaseEParms::CheckPosValue, JCaseEParms.cpp:283-320) ------------
DC_DEFAULT, DC_FIXED, DC_DEFVALUE, DC_DEFPRC = 0, 1, 2, 3


def parse_pos_value(value: str, isposmin: bool) -> tuple[int, float]:
    """(mode, value) of one posmin/posmax attribute: "default", "default +/- v",
    "default +/- v%" or a fixed coordinate.  The sign must enlarge the domain."""
    v = value.replace(" ", "").replace("\t", "").lower()
    if v == "default":
        return DC_DEFAULT, 0.0
    posdef = max(v.find("default+"), v.find("default-"))
    posprc = v.find("%")
    err = None
    if posdef < 0 and posprc >= 0:
        err = "The use of %"
    if err is None and posdef > 0:
        err = "The use of default"
    if err is None and posprc >= 0 and posprc != len(v) - 1:
        err = "The use of %"
    if err is None and posdef == 0 and len(v) <= len("default+"):
        err = "The use of default"
    if err is None:
        if posdef == 0:
            sign = v[7]
            prc = posprc >= 0
            if (isposmin and sign == "+") or (not isposmin and sign == "-"):
                err = "The sign + " if isposmin else "The sign - "
                raise CaseError(f"{err}is invalid in {'posmin' if isposmin else 'posmax'}=\"{value}\" "
                                "to increase the domain.")
            mode = DC_DEFPRC if prc else DC_DEFVALUE
            num = v[8:len(v) - (1 if prc else 0)]
        else:
            mode, num = DC_FIXED, v
        try:
            return mode, float(num)
        except ValueError:
            err = "Number"
    raise CaseError(f"{err} is invalid in {'posmin' if isposmin else 'posmax'}=\"{value}\"")


class _Params:
    """<parameters> as a key -> string map (JCaseEParms)."""

    def __init__(self, node):
        self.values: dict[str, str] = {}
        self.posmin = ["default"] * 3
        self.posmax = ["default"] * 3
        if node is None:
            return
        for e in node.findall("parameter"):
            key, val = e.get("key"), e.get("value")
            if key is None or val is None:
                raise CaseError("A <parameter> needs key and value attributes.")
            if val.startswith("#") and ":" not in val:
                raise CaseError(f"Parameter {key}: user expressions ('#...') are not supported.")
            self.values[key] = val
        dom = node.find("simulationdomain")
        if dom is not None:
            for tag, lst, ismin in (("posmin", self.posmin, True), ("posmax", self.posmax, False)):
                e = dom.find(tag)
                for i, ax in enumerate("xyz"):
                    lst[i] = (e.get(ax) if e is not None else None) or "default"
                    parse_pos_value(lst[i], ismin)  # validates

    def exists(self, key: str) -> bool:
        return key in self.values

    def num(self, key: str, optional: bool = False, default: float = 0.0) -> float:
        if key not in self.values:
            if optional:
                return default
            raise CaseError(f"The parameter '{key}' is missing.")
        s = self.values[key]
        try:
            return float(s)
        except ValueError:
            raise CaseError(f"The parameter '{key}' is not a number: {s!r}") from None

    def int(self, key: str, optional: bool = False, default: int = 0) -> int:
        return int(self.num(key, optional, default))

    def is_pos_default(self) -> bool:
        return all(parse_pos_value(v, True)[0] == DC_DEFAULT for v in self.posmin) and all(
            parse_pos_value(v, False)[0] == DC_DEFAULT for v in self.posmax)


# ---- domain configuration (JSph.cpp:334-427, 1354-1387) ----------------------------------
class _DomainCfg:
    def __init__(self):
        self.clear()

    def clear(self):
        self.pmin = [DBL_MAX] * 3   # CfgDomainParticlesMin
        self.pmax = [DBL_MAX] * 3
        self.prcmin = [DBL_MAX] * 3  # CfgDomainParticlesPrcMin
        self.prcmax = [DBL_MAX] * 3
        self.fmin = [DBL_MAX] * 3   # CfgDomainFixedMin
        self.fmax = [DBL_MAX] * 3

    def resize(self, rmin, rmax, simulate2d: bool) -> tuple[list, list]:
        """JSph::ResizeMapLimits without periodicity and symmetry."""
        if simulate2d:
            for lst in (self.pmin, self.pmax, self.prcmin, self.prcmax, self.fmin, self.fmax):
                lst[1] = DBL_MAX
        dflt = lambda lst, d: [d[i] if lst[i] == DBL_MAX else lst[i] for i in range(3)]  # noqa: E731
        pmin, pmax = dflt(self.pmin, [0.0] * 3), dflt(self.pmax, [0.0] * 3)
        prcmin, prcmax = dflt(self.prcmin, [0.0] * 3), dflt(self.prcmax, [0.0] * 3)
        dif = [rmax[i] - rmin[i] for i in range(3)]
        dmin = [rmin[i] - dif[i] * prcmin[i] for i in range(3)]
        dmax = [rmax[i] + dif[i] * prcmax[i] for i in range(3)]
        dmin = [dmin[i] - pmin[i] for i in range(3)]
        dmax = [dmax[i] + pmax[i] for i in range(3)]
        dmin, dmax = dflt(self.fmin, dmin), dflt(self.fmax, dmax)
        if any(dmin[i] > rmin[i] or dmax[i] < rmax[i] for i in range(3)):
            raise CaseError(f"Domain limits {dmin}-{dmax} are not valid.")
        return dmin, dmax


def _config_domain(p: _Params) -> _DomainCfg:
    """Domain part of JSph::LoadConfigParameters (JSph.cpp:732-756)."""
    d = _DomainCfg()
    resizeold = False
    incz = float(np.float32(p.num("IncZ", True, 0.0)))
    if incz:
        d.clear()
        d.prcmax[2] = incz
        resizeold = True
    if p.exists("DomainFixed"):
        vals = [float(x) for x in p.values["DomainFixed"].split(":")]
        if len(vals) != 6:
            raise CaseError("DomainFixed needs six values xmin:ymin:zmin:xmax:ymax:zmax.")
        d.clear()
        d.fmin, d.fmax = vals[:3], vals[3:]
        resizeold = True
    for key in ("DomainFixedXmin", "DomainFixedYmin", "DomainFixedZmin", "DomainFixedXmax",
                "DomainFixedYmax", "DomainFixedZmax"):
        if p.exists(key):
            ax = "xyz".index(key[-4].lower())
            (d.fmin if key.endswith("min") else d.fmax)[ax] = p.num(key)
            resizeold = True
    if not p.is_pos_default() and resizeold:
        raise CaseError("Combination of <simulationdomain> with IncZ or DomainFixedXXX in <parameters> "
                        "section of XML is not allowed.")
    for i in range(3):
        for ismin, text in ((True, p.posmin[i]), (False, p.posmax[i])):
            mode, v = parse_pos_value(text, ismin)
            if mode == DC_FIXED:
                (d.fmin if ismin else d.fmax)[i] = v
            elif mode == DC_DEFVALUE:
                (d.pmin if ismin else d.pmax)[i] = v
            elif mode == DC_DEFPRC:
                (d.prcmin if ismin else d.prcmax)[i] = v / 100
    return d


# ---- the case -----------------------------------------------------------------------------
# command-line overrides (JSphCfgRun -> JSph::LoadConfigCommands) this core takes
OVERRIDES = ("step_algorithm", "verlet_steps", "tdensity", "ddtvalue", "visco", "viscoboundfactor", "cellmode",
             "celldomfixed", "cflnumber", "rhopoutmin", "rhopoutmax", "timemax", "timeout", "dtini", "dtmin",
             "coefdtmin", "domain_fixed", "tboundary", "slipmode", "mdbc_threshold", "tvisco", "shift_mode",
             "shift_coef", "shift_tfs")


class XmlCase:
    """``<dir>/<name>.xml`` + ``<dir>/<name>.bi4`` (or, with ``partbegin``, the PART
    ``<partbegin_dir>/Part_%04u.bi4``).  Exposes what ``SphGpuSingle`` / ``SphGpuSlab``
    and the PART writer read from a case: ``np, npb, idp, pos, vel, rhop, case_def()``,
    plus the run parameters (``timemax``, ``timeout``, ``time0``, ``symdtpre0``)."""

    def __init__(self, casepath: str, partbegin: int = 0, partbegin_dir: str | None = None, **overrides):
        from .core import read_part  # the .bi4 reader of the core library

        bad = set(overrides) - set(OVERRIDES)
        if bad:
            raise CaseError(f"unknown overrides {sorted(bad)}")
        if casepath.endswith(".xml"):
            casepath = casepath[:-4]
        self.casepath = casepath
        self.case_name = os.path.basename(casepath)
        self._dircase = os.path.dirname(os.path.abspath(casepath))  # JSph::DirCase (data files)
        xmlfile = casepath + ".xml"
        if not os.path.exists(xmlfile):
            raise CaseError(f"Case configuration was not found: {xmlfile}")
        root = ET.parse(xmlfile).getroot()
        if root.tag != "case":
            raise CaseError(f"{xmlfile}: the root element is not <case>.")
        self.app = root.get("app", "unknown")
        ex = _node(root, "execution")
        self._load_constants(_node(ex, "constants"))
        p = _Params(ex.find("parameters"))
        self._load_parameters(p)
        self._domain = _config_domain(p)
        sp = ex.find("special")
        self.phases = ()
        if sp is not None:
            for ch in sp:  # accinputs, chrono, wavepaddles, mlayerpistons, inout, gauges, ...
                if ch.tag == "nnphases" and self.rheology == 2:
                    continue
                raise CaseError(f"<special><{ch.tag}> is not supported by this core.")
        self._load_blocks(_node(ex, "particles"))
        if self.rheology == 2:  # JSph::InitMultiPhase (JSph.cpp:3137-3215 of the v5.0 solver)
            node = sp.find("nnphases") if sp is not None else None
            if node is not None:
                self._load_phases(node)
            else:  # the v5.0 solver would run multiphase without phase data
                raise CaseError("RheologyTreatment=2 needs the phases in <special><nnphases>.")
        self._load_motion(ex.find("motion"))
        dfix = overrides.pop("domain_fixed", None)
        if dfix is not None:  # -domain_fixed: JSph::ConfigDomainFixed (JSph.cpp:343-346, 856)
            self._domain.clear()
            self._domain.fmin, self._domain.fmax = list(dfix[:3]), list(dfix[3:])
        for k, v in overrides.items():
            if k in ("timemax", "timeout") and v < 0 or k == "timemax" and v == 0:
                continue  # JSph::LoadConfigCommands applies TimeMax>0, TimePart>=0 only
            setattr(self, k, v)
        if self.tdensity == 0:
            self.ddtvalue = 0.0
        if not self.rhopoutmin < self.rhopoutmax:  # RhopOut disabled (JSph.cpp:862-863)
            self.rhopoutmin, self.rhopoutmax = -float(np.finfo(np.float32).max), float(np.finfo(np.float32).max)
        if not self.rhopoutmin <= self.rhop0 <= self.rhopoutmax:
            raise CaseError(f"The reference density value {self.rhop0} is outside the defined limits "
                            f"[{self.rhopoutmin},{self.rhopoutmax}].")
        if self.cellmode not in (CELLMODE_FULL, 2):
            raise CaseError("Cell mode is not valid.")
        if self.tboundary == 2 and self.slipmode != 1:  # JSph.cpp:788
            raise CaseError("Only the slip mode velocity=0 is allowed with mDBC conditions.")
        if self.symmetry:  # JSph.cpp:1174-1179
            if self.data2d:
                raise CaseError("Symmetry is not allowed with 2-D simulations.")
            if self.floatings:
                raise CaseError("Symmetry is not allowed with floating bodies.")
            if self.tvisco != 1:
                raise CaseError("Symmetry is only allowed with Artificial viscosity.")
        # -- particles (JPartsLoad4::LoadParticles) ------------------------------------
        self.partbegin = int(partbegin)
        self.partbegin_dir = None
        if self.partbegin:
            d = partbegin_dir if partbegin_dir is not None else os.path.dirname(casepath)
            self.partbegin_dir = d
            fn = os.path.join(d, "Part_%04u.bi4" % self.partbegin)
        else:
            fn = casepath + ".bi4"
        if not os.path.exists(fn):
            raise CaseError(f"File of the particles was not found: {fn}")
        h, prt = read_part(fn)
        self.file_header = h
        self._check_loaded(h, prt)
        self.time0 = float(h["timestep"]) if self.partbegin else 0.0
        self.symdtpre0 = float(h.get("symplectic_dtpre", 0.0)) if self.partbegin else 0.0
        # boundary (fixed + moving) blocks first, stable: the solver's npb leading entries;
        # floating particles sit among the fluid ones (CaseNpb, JSph.cpp)
        isb = prt["idp"] < np.uint32(self.case_npb)
        order = np.concatenate([np.flatnonzero(isb), np.flatnonzero(~isb)])
        self.idp = np.ascontiguousarray(prt["idp"][order], np.uint32)
        self.pos = np.ascontiguousarray(prt["pos"][order], np.float64)
        self.vel = np.ascontiguousarray(prt["vel"][order], np.float32)
        self.rhop = np.ascontiguousarray(prt["rhop"][order], np.float32)
        self.np = int(self.idp.size)
        self.npb = int(isb.sum())
        if self.npb != self.case_npb:
            raise CaseError(f"{fn}: {self.npb} boundary particles loaded, the case has {self.case_npb}.")
        if self.floatings and self.partbegin:
            self._restart_floatings()
        if self.floatings and self.rigidalgorithm != 1:
            raise CaseError("Only RigidAlgorithm=1 (SPH) floating bodies are supported by this core.")
        # case limits (JPartsLoad4 CasePosMin/Max; computed when the file has none)
        cmin, cmax = list(h["case_posmin"]), list(h["case_posmax"])
        if cmin == cmax:
            cmin, cmax = self.pos.min(axis=0).tolist(), self.pos.max(axis=0).tolist()
        self.case_posmin, self.case_posmax = cmin, cmax
        if list(h["map_posmin"]) != list(h["map_posmax"]):
            self._map = (np.array(h["map_posmin"]), np.array(h["map_posmax"]))
        else:
            border = float(np.float32(self.h)) * BORDER_MAP
            rmin = [c - border for c in cmin]
            rmax = [c + border for c in cmax]
            dmin, dmax = self._domain.resize(rmin, rmax, self.data2d)
            if self.symmetry:
                dmin[1] = 0.0  # JSph::ResizeMapLimits (JSph.cpp:1386)
            self._map = (np.array(dmin), np.array(dmax))
        # JSph::CheckRhopLimits (JSph.cpp:2021-2030) is done by the core at creation.
        self._boundnormal = None
        if self.tboundary == 2:
            self._boundnormal = self._load_normals()

    # -- JSphCpu::InitFloating (JSphCpu.cpp:1885-1905) ---------------------------------------
    def _restart_floatings(self) -> None:
        """Restart: every body continues from its state at the PART in PartFloat.fbi4 (center,
        fvel, fomega; the reference starts its angles again from 0)."""
        from .core import read_partfloat

        fn = os.path.join(self.partbegin_dir, "PartFloat.fbi4")
        if not os.path.exists(fn):
            raise CaseError(f"File of floating data was not found: {fn}")
        st = read_partfloat(fn, self.partbegin, len(self.floatings))
        for k, f in enumerate(self.floatings):
            f["center"] = tuple(float(x) for x in st["center"][k])
            f["linvelini"] = tuple(float(x) for x in st["fvel"][k])
            f["angvelini"] = tuple(float(x) for x in st["fomega"][k])

    # -- JSph::LoadBoundNormals (JSph.cpp:1265-1295) ------------------------------------------
    def _load_normals(self) -> np.ndarray:
        from .core import read_extra_normals, read_normals

        out = np.zeros((self.np, 3), np.float32)
        if self.partbegin:
            # JSph::ConfigBoundNormals (JSph.cpp:1308-1316): the normals of the PART from the
            # run's extra data; they are the vectors to the ghost node already, so they are
            # halved here (exact) for the core, which doubles the case file's normals
            fn = os.path.join(self.partbegin_dir, "PartExtra_%04u.bi4" % self.partbegin)
            if not os.path.exists(fn):
                raise CaseError("No extra data available to restart at PART_%04d with mDBC." % self.partbegin)
            nor, useft = read_extra_normals(fn, self.case_nbound, getattr(self, "case_nfloat", 0))
            sel = self.idp < np.uint32(len(nor))
            sel[self.npb:] &= useft  # floating particles only with UseNormalsFt
            out[sel] = nor[self.idp[sel]] * np.float32(0.5)
            if not out[: self.npb].any():
                raise CaseError("No valid normal vectors for using mDBC.")
            return out
        fn = self.casepath + "_Normals.nbi4"
        if os.path.exists(fn):
            nor = read_normals(fn)
            if len(nor) != self.case_nbound:
                raise CaseError(f"{fn}: The number of final normals does not match boundary particles.")
            isb = self.idp < np.uint32(self.case_nbound)
            out[isb] = nor[self.idp[isb]].astype(np.float32)
        elif os.path.exists(self.casepath + "_NormalData.nbi4"):
            raise CaseError("Old normal data file format (XXX_NormalData.nbi4) is invalid for current version.")
        if not out[: self.npb].any():
            raise CaseError("No valid normal vectors for using mDBC.")
        # floating normals (UseNormalsFt, JSph.cpp:1301-1306): mDBC on the floating bodies too
        return out

    @property
    def boundnormal(self) -> np.ndarray | None:
        return self._boundnormal

    # -- JSph::LoadConfigCtes ---------------------------------------------------------------
    def _load_constants(self, c):
        # JCaseCtes::ReadXmlRun (JCaseCtes.cpp:202-204): <data2d> and, when true, <data2dposy>
        self.data2d = _elem_bool(c, "data2d")
        self.data2d_posy = _elem_double(c, "data2dposy") if self.data2d and c.find("data2dposy") is not None else 0.0
        g = c.find("gravity")
        if g is None:
            raise CaseError("The item is not found 'gravity'.")
        self.gravity = tuple(_attr_double(g, a, "gravity") for a in "xyz")
        self.cflnumber = _elem_double(c, "cflnumber")
        self.gamma = _elem_double(c, "gamma")
        self.rhop0 = _elem_double(c, "rhop0")
        self.dp = _elem_double(c, "dp")
        self.h = _elem_double(c, "h")
        self.cteb = _elem_double(c, "b")
        self.massbound = _elem_double(c, "massbound")
        self.massfluid = _elem_double(c, "massfluid")

    # -- JSph::LoadConfigParameters (the keys this core acts on; others refused) -----------
    def _load_parameters(self, p: _Params):
        kern = p.int("Kernel", True, 2)  # JSph.cpp:554-559: 1 Cubic spline, 2 Wendland
        if kern not in (1, 2):
            raise CaseError("Kernel choice is not valid.")
        self.kernel = kern
        # SaveExtraParts (JSph.cpp:598): PART interval (or list) of the mDBC extra data files
        self.sv_extra_parts = p.values.get("SaveExtraParts", "")
        rig = p.int("RigidAlgorithm", True, 1)
        if rig not in (0, 1, 2, 3):
            raise CaseError("Rigid algorithm is not valid.")
        self.rigidalgorithm = rig
        self.ftpause = float(np.float32(p.num("FtPause", True, 0.0)))  # GetValueFloat (JSph.cpp:688)
        self.step_algorithm = p.int("StepAlgorithm", True, 1)
        if self.step_algorithm not in (1, 2):
            raise CaseError("Step algorithm is not valid.")
        self.verlet_steps = p.int("VerletSteps", True, 40)
        # RheologyTreatment / VelocityGradientType / RelaxationDt: the v5.0 NN solver's keys
        # (JSph.cpp:608-623 of src_mphase/DSPH_v5.0_NNewtonian)
        self.rheology = p.int("RheologyTreatment", True, 1)
        if self.rheology not in (1, 2):
            raise CaseError("Rheology treatment is not valid.")
        self.relaxation_dt = float(np.float32(p.num("RelaxationDt", True, 0.2))) if self.rheology == 2 else 0.2
        self.velgrad = p.int("VelocityGradientType", True, 1)
        if self.velgrad not in (1, 2):
            raise CaseError("Velocity gradient treatment is not valid.")
        tv = p.int("ViscoTreatment", True, 1)
        if tv not in (1, 2, 3):
            raise CaseError("Viscosity treatment is not valid.")
        if tv == 3 and self.rheology != 2:
            raise CaseError("ViscoTreatment 'Constitutive  eq.' not valid for Single-phase classic formulation.")
        self.tvisco = tv
        self.visco = p.num("Visco")
        self.viscoboundfactor = p.num("ViscoBoundFactor", True, 1.0)
        # ViscoTime: Visco(t) from a data file next to the case (JDsViscoInput::LoadFile)
        fv = p.values.get("ViscoTime", "")
        self.visco_table = _read_datafile(os.path.join(self._dircase, fv), "ViscoTime") if fv else None
        bc = p.int("Boundary", True, 1)
        if bc not in (1, 2):
            raise CaseError("Boundary Condition method is not valid.")
        self.tboundary = bc
        self.slipmode = 1
        self.mdbc_threshold = 0.0
        self.mdbc_corrector = 0  # JSph.cpp:783: only with mDBC
        if bc == 2:  # JSph.cpp:631-641
            self.slipmode = p.int("SlipMode", True, 1)
            if self.slipmode not in (1, 2, 3):
                raise CaseError("Slip mode is not valid.")
            self.mdbc_corrector = int(p.int("MDBCCorrector", True, 0) != 0)
        if p.exists("DeltaSPH"):
            if p.exists("DensityDT"):
                raise CaseError("The parameters 'DeltaSPH' and 'DensityDT' cannot be combined.")
            v = p.num("DeltaSPH")
            self.tdensity, self.ddtvalue = (1, v) if v > 0 else (0, 0.1)
        else:
            self.tdensity = p.int("DensityDT", True, 0)
            if self.tdensity not in (0, 1, 2, 3):
                raise CaseError("Density Diffusion Term mode is not valid.")
            self.ddtvalue = p.num("DensityDTvalue", True, 0.1)
        self.shift_mode, self.shift_coef, self.shift_tfs = 0, -2.0, 0.0
        if p.exists("Shifting"):  # JSph.cpp:684-700; JSphShifting::ConfigBasic
            sm = p.int("Shifting", True, 0)
            if sm not in (0, 1, 2, 3):
                raise CaseError("Shifting mode in <execution><parameters> is not valid.")
            coef = float(np.float32(p.num("ShiftCoef", True, -2)))
            if sm != 0 and coef != 0:
                self.shift_mode, self.shift_coef = sm, coef
                self.shift_tfs = float(np.float32(p.num("ShiftTFS", True, 0)))
        self.timemax = p.num("TimeMax")
        self.timeout = p.num("TimeOut")
        self.dtini = max(0.0, p.num("DtIni", True, 0.0))
        self.dtmin = max(0.0, p.num("DtMin", True, 0.0))
        self.coefdtmin = p.num("CoefDtMin", True, 0.05)
        self.dtallparticles = 1 if p.int("DtAllParticles", True, 0) == 1 else 0  # JSph.cpp:697
        self.dtfixed = max(0.0, p.num("DtFixed", True, 0.0))  # JSph.cpp:699-707
        ff = p.values.get("DtFixedFile", "")
        ff = "" if ff.upper() == "NONE" else ff
        if self.dtfixed and ff:
            raise CaseError("The parameters 'DtFixed' and 'DtFixedFile' cannot be used at the same time.")
        self.dtfixed_table = _read_datafile(os.path.join(self._dircase, ff), "DtFixedFile") if ff else None
        self.rhopoutmin = p.num("RhopOutMin") if p.exists("RhopOutMin") else 700.0
        self.rhopoutmax = p.num("RhopOutMax") if p.exists("RhopOutMax") else 1300.0
        self.partsoutmax = p.num("PartsOutMax", True, 1.0)
        self.symmetry = p.int("Symmetry", True, 0) != 0  # JSph.cpp:714 (checks: JSph::ConfigBoundary)
        for k in ("XPeriodicIncY", "XPeriodicIncZ", "YPeriodicIncX", "YPeriodicIncZ", "ZPeriodicIncX",
                  "ZPeriodicIncY", "XYPeriodic", "XZPeriodic", "YZPeriodic"):
            if p.exists(k):
                raise CaseError("Periodic boundaries are not supported by this core.")
        self.cellmode = CELLMODE_FULL   # JSphCfgRun default for the GPU (-cellmode:full)
        self.celldomfixed = False

    # -- JCaseParts + JSphMk::Config ---------------------------------------------------------
    def _load_blocks(self, node):
        self.mkboundfirst = int(node.get("mkboundfirst", 11))
        self.mkfluidfirst = int(node.get("mkfluidfirst", 1))
        blocks = []
        for e in node:
            if e.tag not in ("fixed", "moving", "floating", "fluid"):
                if e.tag == "properties" or e.tag.startswith("_") or e.tag == "summary":
                    continue
                raise CaseError(f"<particles>: unknown block <{e.tag}>.")
            b = dict(type=e.tag, mk=int(e.get("mk")), begin=int(e.get("begin")), count=int(e.get("count")),
                     mktype=int(e.get("mkfluid") if e.tag == "fluid" else e.get("mkbound")))
            if e.tag == "floating":
                b["floating"] = self._load_floating(e, self._dircase)
            blocks.append(b)
        kinds = ("fixed", "moving", "floating", "fluid")
        bytype = {k: [b for b in blocks if b["type"] == k] for k in kinds}
        if [b["type"] for b in blocks] != [k for k in kinds for _ in bytype[k]]:
            raise CaseError("<particles>: blocks must be ordered fixed, moving, floating, fluid.")
        begin = 0
        for b in blocks:
            if b["begin"] != begin:
                raise CaseError("<particles>: blocks must be contiguous in idp.")
            begin += b["count"]
        # JSphMk::Config codes: the block index within its type (JSphMk.cpp:108-114)
        base = {"fixed": CODE_TYPE_FIXED, "moving": CODE_TYPE_MOVING, "floating": CODE_TYPE_FLOATING,
                "fluid": CODE_TYPE_FLUID}
        for k in kinds:
            for i, b in enumerate(bytype[k]):
                b["code"] = base[k] | i
        self.blocks = blocks
        self.case_np = begin
        self.case_nfixed = sum(b["count"] for b in bytype["fixed"])
        self.case_nmoving = sum(b["count"] for b in bytype["moving"])
        self.case_nfloat = sum(b["count"] for b in bytype["floating"])
        self.case_npb = self.case_nfixed + self.case_nmoving
        self.case_nbound = self.case_npb + self.case_nfloat
        self.case_nfluid = sum(b["count"] for b in bytype["fluid"])
        self.moving_blocks = bytype["moving"]
        self.floatings = [dict(b["floating"], idbegin=b["begin"], count=b["count"], mkbound=b["mktype"])
                          for b in bytype["floating"]]

    # -- JSph::InitMultiPhase (JSph.cpp:3137-3215, v5.0 NN solver) -----------------------------
    def _load_phases(self, node):
        known = {"rhop", "csound", "gamma", "visco", "tau_yield", "tau_max", "Bi_multi", "HBP_n", "HBP_m",
                 "cohesion", "phi", "phasetype"}
        phases = []
        for e in node:
            if e.tag != "phase":
                if e.tag.startswith("_"):
                    continue
                raise CaseError(f"<nnphases>: unknown element <{e.tag}>.")
            for ch in e:
                if ch.tag not in known and not ch.tag.startswith("_"):
                    raise CaseError(f"<phase>: unknown element <{ch.tag}>.")

            def val(name, optional=False):
                x = e.find(name)
                if x is None:
                    if optional:
                        return 0.0
                    raise CaseError(f"<phase>: the item is not found '{name}'.")
                return float(np.float32(float(x.get("value"))))  # ReadElementFloat

            mkf = int(e.get("mkfluid"))
            if not any(b["type"] == "fluid" and b["mktype"] == mkf for b in self.blocks):
                raise CaseError("No particles with mkfluid=%d" % mkf)
            taumax = val("tau_max", True)
            phases.append(dict(mkfluid=mkf, phasetype=int(val("phasetype")), rho=val("rhop"), cs0=val("csound", True),
                               gamma=val("gamma", True), visco=val("visco"), tau_yield=val("tau_yield"),
                               tau_max=taumax, bi_multi=val("Bi_multi") if taumax else 0.0, hbp_m=val("HBP_m"),
                               hbp_n=val("HBP_n")))
        if not phases:
            raise CaseError("The number of phases is invalid.")
        phases.sort(key=lambda ph: ph["mkfluid"])  # sorted by mkfluid (JSph.cpp:3187-3195)
        # a fluid particle's phase is its code value, the index of its fluid block
        fl = [b for b in self.blocks if b["type"] == "fluid"]
        if [b["mktype"] for b in fl] != [ph["mkfluid"] for ph in phases]:
            raise CaseError("Every fluid block needs its <phase>, in mkfluid order.")
        self.phases = tuple(phases)

    @property
    def explicit_codes(self) -> bool:
        """NN multiphase: the core takes the fluid block codes (the phase of each particle)."""
        return self.rheology == 2

    # -- JCasePartBlock_Floating::ReadXml (JCaseParts.cpp:248-290) ------------------------------
    @staticmethod
    def _load_floating(e, casedir: str = ".") -> dict:
        def d3(name, optional=False, default=(0.0, 0.0, 0.0)):
            x = e.find(name)
            if x is None:
                if optional:
                    return tuple(default)
                raise CaseError(f"<floating>: the item is not found '{name}'.")
            return tuple(_attr_double(x, a, name) for a in "xyz")

        f = dict(massbody=_elem_double(e, "massbody"), masspart=_elem_double(e, "masspart"), center=d3("center"))
        ine = e.find("inertia")
        if ine is None:
            raise CaseError("<floating>: the item is not found 'inertia'.")
        if all(ine.get(a) is not None for a in "xyz"):
            v = d3("inertia")
            f["inertia"] = (v[0], 0.0, 0.0, 0.0, v[1], 0.0, 0.0, 0.0, v[2])
        else:  # JXml::ReadElementMatrix3d: <values v11=.. v12=.. ... v33=../>
            vals = ine.find("values")
            src = vals if vals is not None else ine
            f["inertia"] = tuple(_attr_double(src, "v%d%d" % (r, c), "inertia") for r in (1, 2, 3) for c in (1, 2, 3))

        def i3(a, b):
            if e.find(a) is not None and e.find(b) is not None:
                raise CaseError(f"Only '{a}' or '{b}' must be defined.")
            x = e.find(a) if e.find(a) is not None else e.find(b)
            if x is None:
                return (1, 1, 1)
            return tuple(0 if int(float(x.get(k, "1"))) == 0 else 1 for k in "xyz")

        f["translationfree"] = i3("translation", "translationDOF")
        f["rotationfree"] = i3("rotation", "rotationDOF")
        f["linvelini"] = d3("linearvelini" if e.find("linearvelini") is not None else "velini", True)
        f["angvelini"] = d3("angularvelini" if e.find("angularvelini") is not None else "omegaini", True)
        # imposed velocities ("none" components free) and external forces (JCaseParts.cpp:272-285)
        for name, sub, special in (("linearvel", "vel", True), ("angularvel", "vel", True),
                                   ("linearforce", "force", False), ("angularforce", "force", False)):
            tab = XmlCase._load_linear_values(e, name, sub, special, casedir)
            if tab is not None:
                f[name] = tab
        return f

    # -- JLinearValue::ReadXmlValues (JLinearValue.cpp:493-527), attributes time:x:y:z ---------------
    @staticmethod
    def _load_linear_values(e, name, sub, special, casedir):
        x = e.find(name)
        if x is None:
            return None
        if x.get("file"):  # JSph.cpp:1064-1080: LoadFile(DirCase + file), rows in file order
            return _read_datafile(os.path.join(casedir, x.get("file")), f"<{name}>", 3, special)
        rows = []
        for r in x.findall(sub):
            t = _attr_double(r, "time", sub)
            vals = []
            for a in "xyz":
                txt = r.get(a)
                if special:  # "none" or missing -> DBL_MAX (the component is not imposed)
                    vals.append(np.finfo(np.float64).max if txt is None or txt.strip().lower() == "none"
                                else _attr_double(r, a, sub))
                else:
                    if txt is None:
                        raise CaseError(f"<{name}><{sub}>: the attribute '{a}' is not found.")
                    vals.append(_attr_double(r, a, sub))
            rows.append((t,) + tuple(vals))
        if not rows:
            raise CaseError("There are not times.")
        return np.array(rows, np.float64)  # in the XML's order (JLinearValue walks them as they come)

    # -- JMotion::ReadXml (JMotion.cpp:556-700) + JDsMotion::ConfigObjects (JDsMotion.cpp:67-89) --
    MOV_TYPES = {"wait": 1, "mvrect": 2, "mvrectace": 3, "mvrot": 4, "mvrotace": 5, "mvrectsinu": 6, "mvrotsinu": 7,
                 "mvcir": 8, "mvcirace": 9, "mvcirsinu": 10, "mvrectfile": 11, "mvfile": 11, "mvpredef": 11,
                 "mvrotfile": 12, "mvnull": 13}

    def _load_motion(self, node):
        """The motion program as a tree of objects (<obj> virtual, <objreal ref>), depth first:
        motion = {nobj: the moving blocks, objs: [{parent, ref}], movs / evts with `obj` = the
        node index, rows: the file movements' tables, (t, x, y, z) / (t, degrees, 0, 0)}."""
        self.motion = None
        nobj = len(self.moving_blocks)
        if node is None or not len(list(node)):
            if nobj:
                raise CaseError("The number of mobile objects do not match the predefined motions in XML file.")
            return
        objs, movs, evts, rows = [], [], [], []
        deg2rad, rad2deg = 0.017453292519943295769, 57.29577951308232087684
        f32 = lambda v: float(np.float32(v))  # JXml::GetAttributeFloat
        casedir = self._dircase

        def read(ele, parent):
            for m in ele:
                t = m.tag
                if t.startswith("_"):
                    continue
                if t in ("obj", "objreal"):
                    ref = -1
                    if t == "objreal":
                        if m.get("ref") is None:
                            raise CaseError("<motion><objreal>: the attribute 'ref' is not found.")
                        ref = int(m.get("ref"))
                        if any(o["ref"] == ref for o in objs):
                            raise CaseError(f"Cannot add a new object with an existing real reference (ref={ref}).")
                    objs.append(dict(parent=parent, ref=ref))
                    read(m, len(objs) - 1)
                elif t in XmlCase.MOV_TYPES:
                    if parent < 0:
                        raise CaseError("Missing object.")
                    movs.append(self._motion_mov(m, t, parent, rows, casedir, f32, deg2rad, rad2deg))
                elif parent < 0 or t != "begin":
                    raise CaseError(f"<motion>: unknown element <{t}>.")
            if parent >= 0:  # the object's events, after its elements (JMotion.cpp:688-700)
                for b in ele.findall("begin"):
                    evts.append(dict(obj=parent, mov=int(b.get("mov")), start=f32(b.get("start")),
                                     finish=f32(b.get("finish")) if b.get("finish") is not None else -1.0))

        read(node, -1)
        refs = [o["ref"] for o in objs if o["ref"] >= 0]
        if nobj != max(refs, default=-1) + 1:
            raise CaseError("The number of mobile objects do not match the predefined motions in XML file.")
        if sorted(refs) != list(range(len(refs))):
            raise CaseError("Motion references are no consecutives.")
        self.motion = dict(nobj=nobj, objs=objs, movs=movs, evts=evts, rows=rows)

    @staticmethod
    def _motion_mov(m, t, obj, rows, casedir, f32, deg2rad, rad2deg):
        """One movement as JMotion::ReadXml + MovAdd* hold it (JMotion.cpp:198-300,568-680):
        rotation speeds, accelerations and amplitudes in degrees, phases in radians."""
        typ = XmlCase.MOV_TYPES[t]
        mv = dict(obj=obj, id=int(m.get("id")), next=0, type=typ, prev=0, fields=0, data_first=0, data_n=0,
                  duration=0.0, vec=(0.0,) * 3, vec2=(0.0,) * 3, phase=(0.0,) * 3, axisp1=(0.0,) * 3,
                  axisp2=(0.0,) * 3, ref=(0.0,) * 3, ang=0.0, ang2=0.0, ang3=0.0)
        deg = True
        if t != "mvnull":
            mv["duration"] = f32(m.get("duration"))
            mv["next"] = int(m.get("next", 0))
            units = m.get("anglesunits", "degrees")
            if units not in ("degrees", "radians"):
                raise CaseError("<motion>: invalid anglesunits.")
            deg = units == "degrees"
        if t == "wait" and mv["duration"] < 0:
            raise CaseError("Wating times lenght lower than zero are not allowed.")

        def v3(name):
            x = m.find(name)
            if x is None:
                raise CaseError(f"<motion><{t}>: the item is not found '{name}'.")
            return tuple(_attr_double(x, a, name) for a in "xyz")

        def v1(name, attr):
            x = m.find(name)
            if x is None:
                raise CaseError(f"<motion><{t}>: the item is not found '{name}'.")
            return _attr_double(x, attr, name)

        toang = 1.0 if deg else rad2deg  # speeds / accelerations / amplitudes kept in degrees
        if t in ("mvrot", "mvrotace", "mvrotsinu", "mvcir", "mvcirace", "mvcirsinu", "mvrotfile"):
            mv["axisp1"], mv["axisp2"] = v3("axisp1"), v3("axisp2")
        if t in ("mvcir", "mvcirace", "mvcirsinu"):
            mv["ref"] = v3("ref")
        if t == "mvrect":
            mv["vec"] = v3("vel")
        elif t == "mvrectace":
            mv["vec"] = v3("ace")
            mv["prev"] = int(m.find("velini") is None)
            mv["vec2"] = v3("velini") if not mv["prev"] else (0.0,) * 3
        elif t in ("mvrot", "mvcir"):
            mv["ang"] = v1("vel", "ang") * toang
        elif t in ("mvrotace", "mvcirace"):
            mv["ang"] = v1("ace", "ang") * toang
            mv["prev"] = int(m.find("velini") is None)
            mv["ang2"] = (v1("velini", "ang") * toang) if not mv["prev"] else 0.0
        elif t in ("mvrotsinu", "mvcirsinu"):  # ampl in degrees, phase in radians
            mv["ang"] = v1("freq", "v")
            mv["ang2"] = v1("ampl", "v") * toang
            mv["prev"] = int(m.find("phase") is None)
            mv["ang3"] = (v1("phase", "v") * (deg2rad if deg else 1.0)) if not mv["prev"] else 0.0
        elif t == "mvrectsinu":  # MovAddRecSinu: phase in radians
            mv["vec"], mv["vec2"] = v3("freq"), v3("ampl")
            mv["prev"] = int(m.find("phase") is None)
            mv["phase"] = (tuple(x * deg2rad for x in v3("phase")) if deg else v3("phase")) \
                if not mv["prev"] else (0.0,) * 3
        elif t in ("mvrectfile", "mvfile", "mvpredef", "mvrotfile"):
            ef = m.find("file")
            if ef is None or ef.get("name") is None:
                raise CaseError(f"<motion><{t}>: the item is not found 'file'.")
            fn = ef.get("name")
            path = fn if ("/" in fn or "\\" in fn) else os.path.join(casedir, fn)
            if t == "mvrotfile":  # JMotionDataFile::LoadFileAng: time, angle (radians -> degrees)
                tab = _read_datafile_cols(path, f"<motion><{t}>", 2)
                ang = tab[:, 1] if deg else tab[:, 1] * rad2deg
                new = [(float(a), float(b), 0.0, 0.0) for a, b in zip(tab[:, 0], ang)]
                if len(new) < 2:
                    raise CaseError(f"Cannot be less than two angles. ({path})")
            else:  # LoadFilePos: `fields` values per row; x / y / z where given, else 0
                def iattr(name, default=None):
                    v = ef.get(name)
                    if v is None:
                        if default is None:
                            raise CaseError(f"<motion><{t}><file>: the attribute '{name}' is not found.")
                        return default
                    return int(v)

                fields, ft = iattr("fields"), iattr("fieldtime")
                fx, fy, fz = iattr("fieldx", -1), iattr("fieldy", -1), iattr("fieldz", -1)
                if ft < 0:
                    raise CaseError("The 'time' is not defined.")
                if ft >= fields:
                    raise CaseError("the position of field 'time' is invalid.")
                if fx < 0 and fy < 0 and fz < 0:
                    raise CaseError("You need at least one position field.")
                for nm, f in (("x", fx), ("y", fy), ("z", fz)):
                    if f >= fields:
                        raise CaseError(f"the position of field '{nm}' is invalid.")
                tab = _read_datafile_cols(path, f"<motion><{t}>", fields)
                new = [(float(r[ft]), float(r[fx]) if fx >= 0 else 0.0, float(r[fy]) if fy >= 0 else 0.0,
                        float(r[fz]) if fz >= 0 else 0.0) for r in tab]
                if len(new) < 2:
                    raise CaseError(f"Cannot be less than two positions. ({path})")
                mv["fields"] = (fx >= 0) | ((fy >= 0) << 1) | ((fz >= 0) << 2)
            mv["data_first"], mv["data_n"] = len(rows), len(new)
            rows.extend(new)
        return mv

    def _check_loaded(self, h, prt):
        """JPartsLoad4::CheckConfig (JPartsLoad4.cpp:264-300)."""
        if (h["case_np"], h["case_nfixed"], h["case_nmoving"], h["case_nfloat"], h["case_nfluid"]) != (
                self.case_np, self.case_nfixed, self.case_nmoving, self.case_nfloat, self.case_nfluid):
            raise CaseError("Data file does not match the configuration of the case.")
        if bool(h["data2d"]) != self.data2d:
            raise CaseError("Data file does not match the dimension of the case.")
        if h["peri_mode"] not in (0, 96):  # PERI_None, PERI_Unknown (case files)
            raise CaseError("Data file uses periodic boundaries.")

    # -- what the core and the PART writer read -----------------------------------------
    @property
    def nf(self) -> int:
        return self.np - self.npb

    @property
    def code(self) -> np.ndarray:
        c = np.empty(self.np, np.uint16)
        for b in self.blocks:
            sel = (self.idp >= b["begin"]) & (self.idp < b["begin"] + b["count"])
            c[sel] = b["code"]
        return c

    @property
    def has_bodies(self) -> bool:
        """Moving or floating blocks: the core takes the block codes (JSphMk) of the case."""
        return bool(self.case_nmoving or self.case_nfloat)

    @property
    def mass(self) -> float:
        return self.massfluid

    def map_limits(self) -> tuple[np.ndarray, np.ndarray]:
        return self._map

    def dt_cap(self) -> float:
        """Upper bound of every dt the core can compute (JSphGpu::DtVariable:
        dt = CFL*min(sqrt(h/AceMax), h/(max(Cs0,10*VelMax) + h*ViscDtMax)) <= CFL*h/Cs0,
        floored at DtMin), used by the run driver to batch steps between outputs."""
        k = self._derived()
        cap = k["cflnumber"] * k["kernelh"] / k["cs0"]
        if self.dtfixed > 0:  # DtFixed / DtFixedFile replace the computed dt (JSphCpu.cpp:1621)
            cap = self.dtfixed
        elif self.dtfixed_table is not None:
            cap = float(np.max(self.dtfixed_table[:, 1])) / 1000
        return max(cap, k["dtmin"]) * (1 + 1e-9)

    def _derived(self) -> dict:
        from .core import case_derive

        if getattr(self, "_k", None) is None:
            self._k = case_derive(self.case_def())
        return self._k

    def case_def(self) -> dict:
        """Fields of the C ``SphCaseDef`` (include/sphcore.h)."""
        pmin, pmax = self.map_limits()
        return dict(
            dp=self.dp, h=self.h, cteb=self.cteb, rhop0=self.rhop0, gamma=self.gamma,
            massbound=self.massbound, massfluid=self.massfluid, gravity=tuple(self.gravity),
            cflnumber=self.cflnumber, step_algorithm=self.step_algorithm, verlet_steps=self.verlet_steps,
            kernel=self.kernel, tdensity=self.tdensity, visco=self.visco, viscoboundfactor=self.viscoboundfactor,
            ddtvalue=self.ddtvalue, coefdtmin=self.coefdtmin, dtini=self.dtini, dtmin=self.dtmin,
            rhopoutmin=self.rhopoutmin, rhopoutmax=self.rhopoutmax,
            map_realposmin=tuple(float(v) for v in pmin), map_realposmax=tuple(float(v) for v in pmax),
            cellmode=self.cellmode, celldomfixed=int(self.celldomfixed), npb=self.npb, np=self.np,
            tboundary=self.tboundary, slipmode=self.slipmode, mdbc_threshold=self.mdbc_threshold,
            rheology=self.rheology, velgrad=self.velgrad, tvisco=self.tvisco, nphases=len(self.phases),
            phases=self.phases, relaxation_dt=self.relaxation_dt, shift_mode=self.shift_mode,
            shift_coef=self.shift_coef, shift_tfs=self.shift_tfs, data2d=int(self.data2d),
            data2d_posy=self.data2d_posy, dtallparticles=self.dtallparticles, dtfixed=self.dtfixed,
            symmetry=int(self.symmetry), mdbc_corrector=int(self.mdbc_corrector),
        )


def load_case(casepath: str, partbegin: int = 0, partbegin_dir: str | None = None, **overrides) -> XmlCase:
    return XmlCase(casepath, partbegin, partbegin_dir, **overrides)

