"""ctypes mirror of the POD structs in include/sphcore.h (ABI version: SPH_ABI_VERSION below)."""
from __future__ import annotations

import ctypes as C

import numpy as np

SPH_ABI_VERSION = 12

SPH_STATUS = {
    0: "SPH_OK",
    1: "SPH_ERR_ARG",
    2: "SPH_ERR_HIP",
    3: "SPH_ERR_STATE",
    4: "SPH_ERR_DT",
    5: "SPH_ERR_BOUNDOUT",
    6: "SPH_ERR_NOMEM",
    7: "SPH_ERR_UNSUPPORTED",
    8: "SPH_ERR_COMM",
}


SPH_BOUND_DBC, SPH_BOUND_MDBC = 1, 2
SPH_SLIP_VEL0, SPH_SLIP_NOSLIP, SPH_SLIP_FREESLIP = 1, 2, 3
SPH_RHEOLOGY_SINGLE, SPH_RHEOLOGY_NN = 1, 2
SPH_VELGRAD_FDA, SPH_VELGRAD_SPH = 1, 2
SPH_VISCO_ARTIFICIAL, SPH_VISCO_LAMINARSPS, SPH_VISCO_CONSTEQ = 1, 2, 3
SPH_SHIFT_NONE, SPH_SHIFT_NOBOUND, SPH_SHIFT_NOFIXED, SPH_SHIFT_FULL = 0, 1, 2, 3
SPH_MAXPHASES = 8
_CASEDEF_DEFAULTS = {"tboundary": SPH_BOUND_DBC, "slipmode": SPH_SLIP_VEL0, "mdbc_threshold": 0.0,
                     "rheology": SPH_RHEOLOGY_SINGLE, "velgrad": SPH_VELGRAD_FDA, "tvisco": SPH_VISCO_ARTIFICIAL,
                     "nphases": 0, "relaxation_dt": 0.2, "shift_mode": SPH_SHIFT_NONE, "mdbc_corrector": 0,
                     "shift_coef": -2.0, "shift_tfs": 0.0, "phases": (),
                     "data2d": 0, "pad2d": 0, "data2d_posy": 0.0, "dtallparticles": 0, "symmetry": 0,
                     "dtfixed": 0.0}
SPH_TTAB_DTFIXED, SPH_TTAB_VISCO = 0, 1


class SphPhaseDef(C.Structure):
    """One <nnphases><phase> (JSph::InitMultiPhase, JSph.cpp:3137-3215)."""
    _fields_ = [
        ("mkfluid", C.c_int32),
        ("phasetype", C.c_int32),
        ("rho", C.c_double),
        ("cs0", C.c_double),
        ("gamma", C.c_double),
        ("visco", C.c_double),
        ("tau_yield", C.c_double),
        ("tau_max", C.c_double),
        ("bi_multi", C.c_double),
        ("hbp_m", C.c_double),
        ("hbp_n", C.c_double),
    ]


class SphCaseDef(C.Structure):
    _fields_ = [
        ("dp", C.c_double),
        ("h", C.c_double),
        ("cteb", C.c_double),
        ("rhop0", C.c_double),
        ("gamma", C.c_double),
        ("massbound", C.c_double),
        ("massfluid", C.c_double),
        ("gravity", C.c_double * 3),
        ("cflnumber", C.c_double),
        ("step_algorithm", C.c_int),
        ("verlet_steps", C.c_int),
        ("kernel", C.c_int),
        ("tdensity", C.c_int),
        ("visco", C.c_double),
        ("viscoboundfactor", C.c_double),
        ("ddtvalue", C.c_double),
        ("coefdtmin", C.c_double),
        ("dtini", C.c_double),
        ("dtmin", C.c_double),
        ("rhopoutmin", C.c_double),
        ("rhopoutmax", C.c_double),
        ("map_realposmin", C.c_double * 3),
        ("map_realposmax", C.c_double * 3),
        ("cellmode", C.c_int),
        ("celldomfixed", C.c_int),
        ("npb", C.c_uint32),
        ("np", C.c_uint32),
        ("tboundary", C.c_int32),
        ("slipmode", C.c_int32),
        ("mdbc_threshold", C.c_double),
        ("rheology", C.c_int32),
        ("velgrad", C.c_int32),
        ("tvisco", C.c_int32),
        ("nphases", C.c_uint32),
        ("relaxation_dt", C.c_double),
        ("shift_mode", C.c_int32),
        ("mdbc_corrector", C.c_int32),
        ("shift_coef", C.c_double),
        ("shift_tfs", C.c_double),
        ("phases", SphPhaseDef * SPH_MAXPHASES),
        ("data2d", C.c_int32),
        ("pad2d", C.c_int32),
        ("data2d_posy", C.c_double),
        ("dtallparticles", C.c_int32),
        ("symmetry", C.c_int32),
        ("dtfixed", C.c_double),
    ]

    @classmethod
    def from_dict(cls, d: dict) -> "SphCaseDef":
        s = cls()
        for name, ctype in cls._fields_:
            if name not in d and name in _CASEDEF_DEFAULTS:
                v = _CASEDEF_DEFAULTS[name]
            else:
                v = d[name]
            if name == "phases":
                if len(v) > SPH_MAXPHASES:
                    raise ValueError("at most %d phases" % SPH_MAXPHASES)
                for i, ph in enumerate(v):
                    for k, x in ph.items():
                        setattr(s.phases[i], k, x)
                continue
            if isinstance(v, (tuple, list)):
                arr = getattr(s, name)
                for i, x in enumerate(v):
                    arr[i] = x
            else:
                setattr(s, name, v)
        return s


class SphConstants(C.Structure):
    _fields_ = [
        ("kernelh", C.c_float),
        ("kernelsize", C.c_float),
        ("kernelsize2", C.c_float),
        ("awen", C.c_float),
        ("bwen", C.c_float),
        ("cteb", C.c_float),
        ("gamma", C.c_float),
        ("rhopzero", C.c_float),
        ("ovrhopzero", C.c_float),
        ("massfluid", C.c_float),
        ("massbound", C.c_float),
        ("gravity", C.c_float * 3),
        ("eta2", C.c_float),
        ("ddtkh", C.c_float),
        ("ddtgz", C.c_float),
        ("visco", C.c_float),
        ("viscoboundfactor", C.c_float),
        ("rhopoutmin", C.c_float),
        ("rhopoutmax", C.c_float),
        ("scell", C.c_float),
        ("movlimit", C.c_float),
        ("pad0", C.c_float),
        ("cs0", C.c_double),
        ("cflnumber", C.c_double),
        ("dtini", C.c_double),
        ("dtmin", C.c_double),
        ("dp", C.c_double),
        ("tdensity", C.c_int),
        ("step_algorithm", C.c_int),
        ("verlet_steps", C.c_int),
        ("scelldiv", C.c_int),
        ("map_realposmin", C.c_double * 3),
        ("map_realsize", C.c_double * 3),
        ("dom_posmin", C.c_double * 3),
        ("dom_cells", C.c_uint32 * 3),
        ("dom_cellcode", C.c_uint32),
        ("tboundary", C.c_int32),
        ("slipmode", C.c_int32),
        ("mdbc_threshold", C.c_float),
        ("pad1", C.c_uint32),
        ("rheology", C.c_int32),
        ("velgrad", C.c_int32),
        ("tvisco", C.c_int32),
        ("shift_mode", C.c_int32),
        ("nphases", C.c_uint32),
        ("relaxation_dt", C.c_float),
        ("shift_coef", C.c_float),
        ("shift_tfs", C.c_float),
        ("phase_mass", C.c_float * SPH_MAXPHASES),
        ("phase_cteb", C.c_float * SPH_MAXPHASES),
        ("data2d", C.c_int32),
        ("pad3", C.c_int32),
        ("spssmag", C.c_float),
        ("spsblin", C.c_float),
        ("kernel", C.c_int32),
        ("cub_a1", C.c_float),
        ("cub_a2", C.c_float),
        ("cub_aa", C.c_float),
        ("cub_a24", C.c_float),
        ("cub_c1", C.c_float),
        ("cub_d1", C.c_float),
        ("cub_c2", C.c_float),
        ("cub_od_wdeltap", C.c_float),
        ("pad4", C.c_int32),
        ("dtallparticles", C.c_int32),
        ("symmetry", C.c_int32),
        ("dtfixed", C.c_double),
    ]

    def as_dict(self) -> dict:
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            out[name] = list(v) if hasattr(v, "__len__") else v
        return out


class SphRunStats(C.Structure):
    _fields_ = [
        ("time", C.c_double),
        ("last_dt", C.c_double),
        ("sym_dtpre", C.c_double),
        ("nstep", C.c_uint64),
        ("np", C.c_uint32),
        ("npb", C.c_uint32),
        ("npbok", C.c_uint32),
        ("nout", C.c_uint32),
        ("dtmodif", C.c_uint32),
        ("error_flags", C.c_uint32),
        ("velmax", C.c_float),
        ("acemax", C.c_float),
        ("viscdtmax", C.c_float),
        ("viscetadtmax", C.c_float),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class SphParticlesHost(C.Structure):
    _fields_ = [
        ("n", C.c_uint32),
        ("idp", C.POINTER(C.c_uint32)),
        ("pos", C.POINTER(C.c_double)),
        ("vel", C.POINTER(C.c_float)),
        ("rhop", C.POINTER(C.c_float)),
        ("code", C.POINTER(C.c_uint16)),
        ("boundnormal", C.POINTER(C.c_float)),
    ]


class SphInterOut(C.Structure):
    _fields_ = [
        ("ar", C.POINTER(C.c_float)),
        ("ace", C.POINTER(C.c_float)),
        ("viscdtmax", C.c_float),
        ("velmax", C.c_float),
        ("acemax", C.c_float),
    ]


class SphSlabDef(C.Structure):
    _fields_ = [
        ("rank", C.c_int32),
        ("nranks", C.c_int32),
        ("cx_begin", C.c_int32),
        ("cx_end", C.c_int32),
        ("axis", C.c_int32),
        ("pad", C.c_int32),
        ("comm_id", C.c_ubyte * 128),
    ]


class SphSlabInfo(C.Structure):
    _fields_ = [
        ("rank", C.c_int32),
        ("nranks", C.c_int32),
        ("cx_begin", C.c_int32),
        ("cx_end", C.c_int32),
        ("repartitions", C.c_uint32),
        ("axis", C.c_int32),
        ("last_imbalance", C.c_double),
    ]


class SphPartHeader(C.Structure):
    _fields_ = [
        ("app_name", C.c_char * 64),
        ("case_name", C.c_char * 64),
        ("cpart", C.c_uint32),
        ("npok", C.c_uint32),
        ("nout", C.c_uint32),
        ("step", C.c_uint32),
        ("timestep", C.c_double),
        ("runtime", C.c_double),
        ("domain_min", C.c_double * 3),
        ("domain_max", C.c_double * 3),
        ("symplectic_dtpre", C.c_double),
        ("np_total", C.c_uint64),
        ("case_np", C.c_uint64),
        ("case_nfixed", C.c_uint64),
        ("case_nmoving", C.c_uint64),
        ("case_nfloat", C.c_uint64),
        ("case_nfluid", C.c_uint64),
        ("dp", C.c_double),
        ("h", C.c_double),
        ("b", C.c_double),
        ("rhop0", C.c_double),
        ("gamma", C.c_double),
        ("massbound", C.c_double),
        ("massfluid", C.c_double),
        ("map_posmin", C.c_double * 3),
        ("map_posmax", C.c_double * 3),
        ("case_posmin", C.c_double * 3),
        ("case_posmax", C.c_double * 3),
        ("peri_xinc", C.c_double * 3),
        ("peri_yinc", C.c_double * 3),
        ("peri_zinc", C.c_double * 3),
        ("data2d_posy", C.c_double),
        ("data2d", C.c_int32),
        ("peri_mode", C.c_int32),
        ("axis_div", C.c_int32),
        ("np_dynamic", C.c_int32),
        ("reuse_ids", C.c_int32),
        ("symmetry", C.c_int32),
        ("splitting", C.c_int32),
        ("pos_double", C.c_int32),
        ("visco_type", C.c_int32),
        ("visco", C.c_float),
        ("viscoboundfactor", C.c_float),
        ("gravity", C.c_float * 3),
        ("mkbound", C.c_uint32),
        ("mkfluid", C.c_uint32),
    ]

    def as_dict(self) -> dict:
        d = {}
        for name, t in self._fields_:
            v = getattr(self, name)
            if isinstance(v, bytes):
                v = v.decode()
            elif hasattr(v, "__len__"):
                v = list(v)
            d[name] = v
        return d

    @classmethod
    def from_dict(cls, d: dict) -> "SphPartHeader":
        h = cls()
        for name, t in cls._fields_:
            if name not in d:
                continue
            v = d[name]
            if isinstance(v, str):
                v = v.encode()
            if hasattr(getattr(h, name), "__len__") and not isinstance(v, bytes):
                arr = getattr(h, name)
                for i, x in enumerate(v):
                    arr[i] = x
            else:
                setattr(h, name, v)
        return h


def _ptr(arr: np.ndarray | None, ctype):
    if arr is None:
        return C.POINTER(ctype)()
    assert arr.flags["C_CONTIGUOUS"]
    return arr.ctypes.data_as(C.POINTER(ctype))


class SphMotionMov(C.Structure):
    _fields_ = [
        ("obj", C.c_int32), ("id", C.c_int32), ("next", C.c_int32), ("type", C.c_int32), ("prev", C.c_int32),
        ("fields", C.c_int32), ("data_first", C.c_uint32), ("data_n", C.c_uint32), ("duration", C.c_double),
        ("vec", C.c_double * 3), ("vec2", C.c_double * 3), ("phase", C.c_double * 3), ("axisp1", C.c_double * 3),
        ("axisp2", C.c_double * 3), ("ref", C.c_double * 3), ("ang", C.c_double), ("ang2", C.c_double),
        ("ang3", C.c_double),
    ]


class SphMotionObj(C.Structure):
    _fields_ = [("parent", C.c_int32), ("ref", C.c_int32)]


class SphMotionEvent(C.Structure):
    _fields_ = [("obj", C.c_int32), ("mov", C.c_int32), ("start", C.c_double), ("finish", C.c_double)]


class SphFloatingDef(C.Structure):
    _fields_ = [
        ("idbegin", C.c_uint32), ("count", C.c_uint32), ("massbody", C.c_double), ("masspart", C.c_double),
        ("center", C.c_double * 3), ("inertia", C.c_double * 9), ("linvelini", C.c_double * 3),
        ("angvelini", C.c_double * 3), ("translationfree", C.c_int32 * 3), ("rotationfree", C.c_int32 * 3),
    ]


class SphFloatingState(C.Structure):
    _fields_ = [
        ("center", C.c_double * 3), ("fvel", C.c_float * 3), ("fomega", C.c_float * 3), ("angles", C.c_float * 3),
        ("facelin", C.c_float * 3), ("faceang", C.c_float * 3), ("pad", C.c_float),
    ]

    def as_dict(self) -> dict:
        return {k: np.array(getattr(self, k)) for k in ("center", "fvel", "fomega", "angles", "facelin", "faceang")}


def _fill(struct, d: dict):
    for k, v in d.items():
        if k not in dict(struct._fields_):
            continue
        f = getattr(struct, k)
        if isinstance(f, C.Array):
            for i, x in enumerate(v):
                f[i] = x
        else:
            setattr(struct, k, v)
    return struct


def motion_arrays(motion: dict):
    """SphMotionMov[] / SphMotionEvent[] of a case's motion program (XmlCase.motion)."""
    movs = (SphMotionMov * max(1, len(motion["movs"])))()
    for i, m in enumerate(motion["movs"]):
        _fill(movs[i], m)
    evts = (SphMotionEvent * max(1, len(motion["evts"])))()
    for i, e in enumerate(motion["evts"]):
        _fill(evts[i], e)
    return movs, evts


def motion_tree_arrays(motion: dict):
    """The tree form (motion["objs"]: nodes depth first with parent / ref; movement and event
    `obj` are node indices; motion["rows"]: the file movements' table rows, 4 doubles each):
    SphMotionObj[], SphMotionMov[], SphMotionEvent[], the rows (float64, C order)."""
    nodes = (SphMotionObj * len(motion["objs"]))()
    for i, o in enumerate(motion["objs"]):
        nodes[i].parent, nodes[i].ref = int(o["parent"]), int(o["ref"])
    movs, evts = motion_arrays(motion)
    rows = np.ascontiguousarray(np.asarray(motion.get("rows", np.zeros((0, 4))), np.float64).reshape(-1, 4))
    return nodes, movs, evts, rows


def floating_array(floatings: list):
    arr = (SphFloatingDef * len(floatings))()
    for i, f in enumerate(floatings):
        _fill(arr[i], f)
    return arr


class HostParticles:
    """Owns numpy arrays and exposes them as an SphParticlesHost view."""

    def __init__(self, n: int, idp=None, pos=None, vel=None, rhop=None, code=None, boundnormal=None):
        self.idp = np.ascontiguousarray(idp if idp is not None else np.zeros(n, np.uint32), dtype=np.uint32)
        self.pos = np.ascontiguousarray(pos if pos is not None else np.zeros((n, 3)), dtype=np.float64)
        self.vel = np.ascontiguousarray(vel if vel is not None else np.zeros((n, 3), np.float32), dtype=np.float32)
        self.rhop = np.ascontiguousarray(rhop if rhop is not None else np.zeros(n, np.float32), dtype=np.float32)
        self.code = np.ascontiguousarray(code if code is not None else np.zeros(n, np.uint16), dtype=np.uint16)
        self.boundnormal = (None if boundnormal is None
                            else np.ascontiguousarray(boundnormal, dtype=np.float32).reshape(n, 3))
        self.view = SphParticlesHost(
            n,
            _ptr(self.idp, C.c_uint32),
            _ptr(self.pos, C.c_double),
            _ptr(self.vel, C.c_float),
            _ptr(self.rhop, C.c_float),
            _ptr(self.code, C.c_uint16),
            _ptr(self.boundnormal, C.c_float),
        )

    def trimmed(self, n: int) -> dict:
        return dict(
            idp=self.idp[:n].copy(),
            pos=self.pos[:n].copy(),
            vel=self.vel[:n].copy(),
            rhop=self.rhop[:n].copy(),
            code=self.code[:n].copy(),
        )


def check_struct_sizes() -> dict:
    return {
        "SphCaseDef": C.sizeof(SphCaseDef),
        "SphConstants": C.sizeof(SphConstants),
        "SphRunStats": C.sizeof(SphRunStats),
        "SphParticlesHost": C.sizeof(SphParticlesHost),
        "SphInterOut": C.sizeof(SphInterOut),
        "SphSlabDef": C.sizeof(SphSlabDef),
        "SphPartHeader": C.sizeof(SphPartHeader),
        "SphMotionMov": C.sizeof(SphMotionMov),
        "SphMotionEvent": C.sizeof(SphMotionEvent),
        "SphFloatingDef": C.sizeof(SphFloatingDef),
        "SphFloatingState": C.sizeof(SphFloatingState),
    }
