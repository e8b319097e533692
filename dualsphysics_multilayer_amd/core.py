"""Host-side mirror of the reference solver interface over the HIP core (C-ABI).

``SphGpuSingle`` follows ``JSphGpuSingle`` (JSphGpuSingle.h:35): the same phase
names (``RunCellDivide``, ``Interaction_Forces``, ``DtVariable``,
``ComputeVerlet``, ``ComputeSymplecticPre/Corr``, ``ComputeStep``, ``Run``),
the same fail-fast behaviour (a non-zero status raises ``SphError`` carrying the
core's message, as ``Check_CudaErroor`` raises ``JException``,
RunExceptionGpuDef.h:27) and the same data out (``ParticlesDataDown`` feeding
SaveData).  Everything executes in ``libsphcore.so``; there is no CPU fallback:
if the library or a HIP device is missing, construction raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._abi import (
    SPH_ABI_VERSION,
    SPH_TTAB_DTFIXED,
    SPH_TTAB_VISCO,
    SPH_STATUS,
    HostParticles,
    SphCaseDef,
    SphConstants,
    SphInterOut,
    SphRunStats,
    SphPartHeader,
    SphSlabDef,
    SphSlabInfo,
    SphFloatingDef,
    SphFloatingState,
    SphMotionEvent,
    SphMotionMov,
    SphMotionObj,
    floating_array,
    motion_arrays,
    motion_tree_arrays,
)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPH_LIB") or os.path.join(HERE, "lib", "libsphcore.so")

INTERSTEP_VERLET, INTERSTEP_SYMPREDICTOR, INTERSTEP_SYMCORRECTOR = 1, 2, 3

EXPORTED_SYMBOLS = (
    "sph_abi_version",
    "sph_last_error",
    "sph_case_derive",
    "sph_solver_create",
    "sph_solver_destroy",
    "sph_divide",
    "sph_interaction_forces",
    "sph_compute_dt",
    "sph_step_verlet",
    "sph_step_symplectic_pre",
    "sph_step_symplectic_cor",
    "sph_solver_run",
    "sph_solver_sync",
    "sph_solver_stats",
    "sph_solver_dt_trace",
    "sph_download_particles",
    "sph_download_interaction",
    "sph_count_pairs",
    "sph_solver_set_time",
    "sph_solver_set_timing",
    "sph_solver_set_timing_phases",
    "sph_solver_timing",
    "sph_slab_partition",
    "sph_slab_partition_axis",
    "sph_comm_unique_id",
    "sph_slab_create",
    "sph_slab_create_shm",
    "sph_slab_group_create",
    "sph_slab_group_create_axis",
    "sph_slab_group_destroy",
    "sph_slab_group_run",
    "sph_slab_group_member",
    "sph_slab_set_repartition",
    "sph_slab_group_set_repartition",
    "sph_slab_set_overlap",
    "sph_slab_group_set_overlap",
    "sph_slab_info",
    "sph_part_read",
    "sph_part_write",
    "sph_part_head_write",
    "sph_normals_read",
    "sph_normals_write",
    "sph_bi4_rewrite",
    "sph_solver_set_motion",
    "sph_solver_set_motion_tree",
    "sph_solver_set_floatings",
    "sph_solver_set_floating_table",
    "sph_solver_set_time_table",
    "sph_solver_floatings",
    "sph_partfloat_write",
    "sph_partfloat_read",
    "sph_extra_normals_read",
    "sph_extra_normals_write",
    "sph_download_normals",
)


# <floating> tables of a body, in SPH_FTTAB_* order (sphcore.h)
FT_TABLES = ("linearvel", "angularvel", "linearforce", "angularforce")


class SphError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__("%s: %s" % (SPH_STATUS.get(status, status), msg))
        self.status = status


_lib = None


def load_library(path: str = LIB_PATH):
    """Loads libsphcore.so (no compute happens here; works without a GPU)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SphError(3, "HIP core %s is not built (run __graft_entry__.build())" % path)
    L = C.CDLL(path)
    vp = C.c_void_p
    L.sph_abi_version.restype = C.c_int
    L.sph_last_error.restype = C.c_char_p
    L.sph_case_derive.argtypes = [C.POINTER(SphCaseDef), C.POINTER(SphConstants)]
    L.sph_solver_create.argtypes = [C.POINTER(SphCaseDef), vp, C.c_int, C.POINTER(vp)]
    for name in ("sph_solver_destroy", "sph_divide", "sph_step_verlet", "sph_step_symplectic_pre",
                 "sph_step_symplectic_cor", "sph_solver_sync"):
        getattr(L, name).argtypes = [vp]
    L.sph_interaction_forces.argtypes = [vp, C.c_int]
    L.sph_compute_dt.argtypes = [vp, C.c_int]
    L.sph_solver_run.argtypes = [vp, C.c_uint32]
    L.sph_solver_stats.argtypes = [vp, C.POINTER(SphRunStats)]
    L.sph_solver_dt_trace.argtypes = [vp, C.POINTER(C.c_double), C.c_uint32, C.POINTER(C.c_uint32)]
    L.sph_download_particles.argtypes = [vp, vp]
    L.sph_download_interaction.argtypes = [vp, C.POINTER(SphInterOut)]
    L.sph_count_pairs.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.sph_solver_set_timing.argtypes = [vp, C.c_int]
    L.sph_solver_set_timing_phases.argtypes = [vp, C.c_uint]
    L.sph_solver_set_time.argtypes = [vp, C.c_double, C.c_double]
    L.sph_solver_timing.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
    L.sph_slab_partition.argtypes = [C.POINTER(SphCaseDef), vp, C.c_int, C.c_double, C.POINTER(C.c_int32)]
    L.sph_slab_partition_axis.argtypes = [C.POINTER(SphCaseDef), vp, C.c_int, C.c_double, C.c_int,
                                          C.POINTER(C.c_int32)]
    L.sph_comm_unique_id.argtypes = [C.POINTER(C.c_ubyte)]
    L.sph_slab_create.argtypes = [C.POINTER(SphCaseDef), vp, C.c_int, C.POINTER(SphSlabDef), C.POINTER(vp)]
    L.sph_slab_create_shm.argtypes = [C.POINTER(SphCaseDef), vp, C.c_int,
                                      C.POINTER(SphSlabDef), C.c_char_p, C.c_uint64, C.POINTER(vp)]
    L.sph_slab_group_create.argtypes = [C.POINTER(SphCaseDef), vp, C.c_int, C.POINTER(C.c_int32),
                                        C.POINTER(C.c_int32), C.POINTER(vp)]
    L.sph_slab_group_create_axis.argtypes = [C.POINTER(SphCaseDef), vp, C.c_int, C.POINTER(C.c_int32), C.c_int,
                                             C.POINTER(C.c_int32), C.POINTER(vp)]
    L.sph_slab_group_destroy.argtypes = [vp]
    L.sph_slab_group_run.argtypes = [vp, C.c_uint32]
    L.sph_slab_group_member.argtypes = [vp, C.c_int, C.POINTER(vp)]
    L.sph_slab_set_repartition.argtypes = [vp, C.c_uint32, C.c_double, C.c_double]
    L.sph_slab_group_set_repartition.argtypes = [vp, C.c_uint32, C.c_double, C.c_double]
    L.sph_slab_set_overlap.argtypes = [vp, C.c_int]
    L.sph_slab_group_set_overlap.argtypes = [vp, C.c_int]
    L.sph_slab_info.argtypes = [vp, C.POINTER(SphSlabInfo)]
    L.sph_part_read.argtypes = [C.c_char_p, C.POINTER(SphPartHeader), vp]
    L.sph_part_write.argtypes = [C.c_char_p, C.POINTER(SphPartHeader), vp]
    L.sph_bi4_rewrite.argtypes = [C.c_char_p, C.c_char_p]
    L.sph_part_head_write.argtypes = [C.c_char_p, C.POINTER(SphPartHeader)]
    L.sph_normals_read.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_double), C.POINTER(C.c_uint32)]
    L.sph_normals_write.argtypes = [C.c_char_p, C.c_char_p, C.c_double, C.c_double, C.c_double, C.c_uint32,
                                    C.POINTER(C.c_double)]
    L.sph_solver_set_motion.argtypes = [vp, C.c_uint32, C.c_uint32, C.POINTER(SphMotionMov), C.c_uint32,
                                        C.POINTER(SphMotionEvent)]
    L.sph_solver_set_motion_tree.argtypes = [vp, C.c_uint32, C.POINTER(SphMotionObj), C.c_uint32,
                                             C.POINTER(SphMotionMov), C.c_uint32, C.POINTER(SphMotionEvent),
                                             C.c_uint32, C.POINTER(C.c_double)]
    L.sph_solver_set_floatings.argtypes = [vp, C.c_uint32, C.POINTER(SphFloatingDef), C.c_double]
    L.sph_solver_set_time_table.argtypes = [vp, C.c_int32, C.c_uint32, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.sph_solver_set_floating_table.argtypes = [vp, C.c_uint32, C.c_int32, C.c_uint32, C.POINTER(C.c_double),
                                                C.POINTER(C.c_double)]
    L.sph_solver_floatings.argtypes = [vp, C.c_uint32, C.POINTER(SphFloatingState), C.POINTER(C.c_uint32)]
    L.sph_partfloat_write.argtypes = [C.c_char_p, C.c_char_p, C.c_uint32, C.c_uint32] + [vp] * 6 + [C.c_uint32] + [vp] * 8
    L.sph_partfloat_read.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32, vp, vp, vp, vp]
    L.sph_extra_normals_read.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, vp, C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_int32)]
    L.sph_extra_normals_write.argtypes = [C.c_char_p, C.c_char_p, C.c_uint32, C.c_uint32, C.c_double, C.c_uint32,
                                          C.c_uint32, C.c_int32, C.c_uint32, vp]
    L.sph_download_normals.argtypes = [vp, C.c_uint32, vp, C.POINTER(C.c_uint32), C.POINTER(C.c_int32)]
    if L.sph_abi_version() != SPH_ABI_VERSION:
        raise SphError(3, "ABI version mismatch")
    _lib = L
    return L


def _check(r: int) -> None:
    if r != 0:
        raise SphError(r, load_library().sph_last_error().decode())


def case_derive(case_def: dict) -> dict:
    """JSph::ConfigConstants1/2 + cell division through the core (no GPU needed)."""
    k = SphConstants()
    _check(load_library().sph_case_derive(C.byref(SphCaseDef.from_dict(case_def)), C.byref(k)))
    return k.as_dict()


def case_particles(case) -> HostParticles:
    """Initial particles of a case; the particle codes travel only when the case has moving or
    floating blocks (else the core assigns one fixed + one fluid block, JSph::LoadCodeParticles)."""
    bodies = getattr(case, "has_bodies", False) or getattr(case, "explicit_codes", False)
    hp = HostParticles(case.np, case.idp, case.pos, case.vel, case.rhop, code=case.code if bodies else None,
                       boundnormal=getattr(case, "boundnormal", None))
    if not bodies:
        hp.view.code = C.POINTER(C.c_uint16)()
    return hp


class SphGpuSingle:
    """One MI355X running one domain: the JSphGpuSingle of this core."""

    def __init__(self, case, device: int = 0):
        L = load_library()
        self.case = case
        self._cdef = SphCaseDef.from_dict(case.case_def())
        init = case_particles(case)
        h = C.c_void_p()
        _check(L.sph_solver_create(C.byref(self._cdef), C.byref(init.view), device, C.byref(h)))
        self._h = h
        self._time_set = None
        self._configure_bodies()

    def set_time_table(self, kind: int, rows) -> None:
        """DtFixedFile (kind SPH_TTAB_DTFIXED: rows (time s, dt ms)) or ViscoTime (SPH_TTAB_VISCO:
        rows (time, Visco)) of the step; None / empty removes the table."""
        rows = np.zeros((0, 2)) if rows is None else np.ascontiguousarray(rows, np.float64).reshape(-1, 2)
        t, v = np.ascontiguousarray(rows[:, 0]), np.ascontiguousarray(rows[:, 1])
        dp = C.POINTER(C.c_double)
        _check(load_library().sph_solver_set_time_table(self._h, kind, len(rows), t.ctypes.data_as(dp),
                                                         v.ctypes.data_as(dp)))

    def _configure_bodies(self) -> None:
        """Time tables, motion program and floating bodies of the case (JSph::LoadCaseConfig)."""
        case, L = self.case, load_library()
        for kind, key in ((SPH_TTAB_DTFIXED, "dtfixed_table"), (SPH_TTAB_VISCO, "visco_table")):
            if getattr(case, key, None) is not None:
                self.set_time_table(kind, getattr(case, key))
        if not getattr(case, "has_bodies", False):
            return
        # a restart sets the PART time first: the motion program is advanced to it
        if getattr(case, "time0", 0.0) or getattr(case, "symdtpre0", 0.0):
            self.set_time(case.time0, case.symdtpre0)
        if getattr(case, "motion", None) and "objs" in case.motion:  # nested objects / file tables
            nodes, movs, evts, rows = motion_tree_arrays(case.motion)
            _check(L.sph_solver_set_motion_tree(self._h, len(case.motion["objs"]), nodes, len(case.motion["movs"]),
                                                movs, len(case.motion["evts"]), evts, len(rows),
                                                rows.ctypes.data_as(C.POINTER(C.c_double))))
        elif getattr(case, "motion", None):
            movs, evts = motion_arrays(case.motion)
            _check(L.sph_solver_set_motion(self._h, case.motion["nobj"], len(case.motion["movs"]), movs,
                                           len(case.motion["evts"]), evts))
        if getattr(case, "floatings", None):
            fts = floating_array(case.floatings)
            _check(L.sph_solver_set_floatings(self._h, len(case.floatings), fts, case.ftpause))
            # imposed velocities / external forces (SPH_FTTAB_* order): rows (time, x, y, z)
            for b, f in enumerate(case.floatings):
                for kind, key in enumerate(FT_TABLES):
                    rows = f.get(key)
                    if rows is None or not len(rows):
                        continue
                    rows = np.ascontiguousarray(rows, np.float64)
                    t, v = np.ascontiguousarray(rows[:, 0]), np.ascontiguousarray(rows[:, 1:4])
                    dp = C.POINTER(C.c_double)
                    _check(L.sph_solver_set_floating_table(self._h, b, kind, len(rows), t.ctypes.data_as(dp),
                                                           v.ctypes.data_as(dp)))

    def close(self) -> None:
        if getattr(self, "_h", None):
            load_library().sph_solver_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- phases (JSphGpuSingle names) --------------------------------------
    def RunCellDivide(self) -> None:
        _check(load_library().sph_divide(self._h))

    def Interaction_Forces(self, interstep: int = INTERSTEP_VERLET) -> None:
        _check(load_library().sph_interaction_forces(self._h, interstep))

    def ComputeVerlet(self) -> None:
        _check(load_library().sph_step_verlet(self._h))

    def ComputeSymplecticPre(self) -> None:
        _check(load_library().sph_step_symplectic_pre(self._h))

    def ComputeSymplecticCorr(self) -> None:
        _check(load_library().sph_step_symplectic_cor(self._h))

    def Run(self, nsteps: int) -> None:
        """nsteps x (ComputeStep + RunCellDivide); asynchronous until sync()."""
        _check(load_library().sph_solver_run(self._h, nsteps))

    run = Run

    def sync(self) -> None:
        _check(load_library().sph_solver_sync(self._h))

    # -- data out ---------------------------------------------------------
    def stats(self) -> dict:
        s = SphRunStats()
        _check(load_library().sph_solver_stats(self._h, C.byref(s)))
        return s.as_dict()

    def dt_trace(self) -> np.ndarray:
        cnt = C.c_uint32()
        _check(load_library().sph_solver_dt_trace(self._h, None, 0, C.byref(cnt)))
        out = np.zeros(cnt.value, np.float64)
        _check(load_library().sph_solver_dt_trace(self._h, out.ctypes.data_as(C.POINTER(C.c_double)), cnt.value,
                                                  C.byref(cnt)))
        return out

    def particles(self) -> dict:
        hp = HostParticles(self.case.np)
        _check(load_library().sph_download_particles(self._h, C.byref(hp.view)))
        return hp.trimmed(hp.view.n)

    def interaction(self) -> dict:
        n = self.stats()["np"]
        ar = np.zeros(n, np.float32)
        ace = np.zeros((n, 3), np.float32)
        out = SphInterOut(ar.ctypes.data_as(C.POINTER(C.c_float)), ace.ctypes.data_as(C.POINTER(C.c_float)), 0, 0, 0)
        _check(load_library().sph_download_interaction(self._h, C.byref(out)))
        return dict(ar=ar, ace=ace, viscdtmax=out.viscdtmax, velmax=out.velmax, acemax=out.acemax)

    def count_pairs(self) -> np.ndarray:
        out = np.zeros(6, np.uint64)
        _check(load_library().sph_count_pairs(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64))))
        return out

    def set_time(self, time: float, symplectic_dtpre: float = 0.0) -> None:
        """Restart from a PART: its TimeStep (and SymplecticDtPre)."""
        if getattr(self, "_time_set", None) == (time, symplectic_dtpre):
            return  # already applied at creation (cases with moving/floating bodies)
        _check(load_library().sph_solver_set_time(self._h, time, symplectic_dtpre))
        self._time_set = (time, symplectic_dtpre)

    def normals(self) -> tuple[np.ndarray, bool]:
        """mDBC: the current vectors particle -> ghost node by idp, and UseNormalsFt."""
        L = load_library()
        n, ft = C.c_uint32(), C.c_int32()
        _check(L.sph_download_normals(self._h, 0, None, C.byref(n), C.byref(ft)))
        out = np.zeros((n.value, 3), np.float32)
        _check(L.sph_download_normals(self._h, n.value, out.ctypes.data, C.byref(n), C.byref(ft)))
        return out, bool(ft.value)

    def floatings(self) -> list:
        """State of the floating bodies (FtObjs: center, fvel, fomega, angles, facelin, faceang)."""
        n = C.c_uint32()
        _check(load_library().sph_solver_floatings(self._h, 0, None, C.byref(n)))
        out = (SphFloatingState * max(1, n.value))()
        _check(load_library().sph_solver_floatings(self._h, n.value, out, C.byref(n)))
        return [out[i].as_dict() for i in range(n.value)]

    def save_part(self, path: str, cpart: int, head_path: str | None = None) -> None:
        """SaveData: this solver's state as a reference PART file (+ Part_Head.ibi4)."""
        p = self.particles()  # solver (cell-sorted) order, as the reference saves
        hdr = part_header(self.case, self.stats(), cpart)
        write_part(path, hdr, {k: p[k] for k in ("idp", "pos", "vel", "rhop")})
        if head_path:
            write_part_head(head_path, hdr)

    def set_timing(self, on: bool, phases: int = 0xF) -> None:
        """Time the next steps' phases (bit i of `phases`: phase i of timing(); all by default)."""
        _check(load_library().sph_solver_set_timing_phases(self._h, int(phases)))
        _check(load_library().sph_solver_set_timing(self._h, int(on)))

    def slab_info(self) -> dict:
        """Current owned cells of a slab (along its axis), re-partitions so far, last measured imbalance."""
        out = SphSlabInfo()
        _check(load_library().sph_slab_info(self._h, C.byref(out)))
        return {k: getattr(out, k) for k, _ in SphSlabInfo._fields_ if k != "pad"}

    def set_repartition(self, every: int, bound_weight: float = 0.3, tolerance: float = 0.05) -> None:
        """Slabs: re-balance the column bounds every `every` steps (collective)."""
        _check(load_library().sph_slab_set_repartition(self._h, every, bound_weight, tolerance))

    def set_overlap(self, on: bool) -> None:
        """Slabs: send a divide's ghost records beside the interaction of the items that
        need none (default on; the results are bitwise the same either way)."""
        _check(load_library().sph_slab_set_overlap(self._h, int(on)))

    def timing(self) -> tuple[np.ndarray, int]:
        ms = np.zeros(4, np.float64)
        n = C.c_uint64()
        _check(load_library().sph_solver_timing(self._h, ms.ctypes.data_as(C.POINTER(C.c_double)), C.byref(n)))
        return ms, n.value


# ---- slab decomposition over x or y --------------------------------
def slab_partition(case, nranks: int, bound_weight: float = 0.3, axis: int = 0) -> np.ndarray:
    """Cell bounds [nranks+1] along `axis` (0: x columns, 1: y rows) balancing
    fluid + bound_weight*bound particles."""
    cdef = SphCaseDef.from_dict(case.case_def())
    init = case_particles(case)
    out = np.zeros(nranks + 1, np.int32)
    _check(load_library().sph_slab_partition_axis(C.byref(cdef), C.byref(init.view), nranks, bound_weight, int(axis),
                                                  out.ctypes.data_as(C.POINTER(C.c_int32))))
    return out


def comm_unique_id() -> bytes:
    """RCCL bootstrap id (rank 0 creates it, the host broadcasts it to every rank)."""
    buf = (C.c_ubyte * 128)()
    _check(load_library().sph_comm_unique_id(buf))
    return bytes(buf)


class SphGpuSlab(SphGpuSingle):
    """One slab of a domain decomposed over x (axis 0) or y (axis 1), one process per GPU
    over RCCL.

    Every rank passes the full case; `bounds` are the cell bounds of all ranks along the
    axis (slab_partition) and `comm_id` the id rank 0 created.  Run/phase calls are
    collective.  stats()["np"] and particles() cover the owned particles only."""

    def __init__(self, case, rank: int, nranks: int, bounds, comm_id, device: int = 0, transport: str = "rccl",
                 slot_bytes: int = 16 << 20, axis: int = 0):
        """transport "rccl": comm_id = comm_unique_id() of rank 0 (one process per GPU);
        "shm": comm_id = the shared-memory segment name ("/...", same on every rank; ranks of
        one node without RCCL, e.g. several on one GPU), slot_bytes per mailbox."""
        L = load_library()
        self.case = case
        self._cdef = SphCaseDef.from_dict(case.case_def())
        init = case_particles(case)
        sd = SphSlabDef(rank, nranks, int(bounds[rank]), int(bounds[rank + 1]), int(axis))
        h = C.c_void_p()
        if transport == "shm":
            _check(L.sph_slab_create_shm(C.byref(self._cdef), C.byref(init.view), device, C.byref(sd),
                                         comm_id.encode() if isinstance(comm_id, str) else comm_id, slot_bytes,
                                         C.byref(h)))
        elif transport == "rccl":
            C.memmove(sd.comm_id, comm_id, 128)
            _check(L.sph_slab_create(C.byref(self._cdef), C.byref(init.view), device, C.byref(sd), C.byref(h)))
        else:
            raise ValueError("transport must be 'rccl' or 'shm'")
        self._h = h
        self._time_set = None
        self.bounds = np.asarray(bounds)
        self.rank = rank
        self._configure_bodies()


class _SlabMember(SphGpuSingle):
    """Borrowed member handle of a SphSlabGroup (data-out calls only)."""

    def __init__(self, group, h, case):
        self.case = case
        self._group = group
        self._h = h
        self._time_set = None

    def close(self) -> None:
        self._h = None


class SphSlabGroup:
    """Several slabs of one domain in ONE process (host threads; devices may repeat).

    Runs the same pack / exchange / reduce code as SphGpuSlab over device-to-device
    copies instead of RCCL — how the decomposition is tested on a one-GPU machine."""

    def __init__(self, case, bounds, devices=None, axis: int = 0):
        L = load_library()
        bounds = np.ascontiguousarray(bounds, np.int32)
        n = len(bounds) - 1
        devices = np.ascontiguousarray(devices if devices is not None else np.zeros(n), np.int32)
        self.case = case
        self._cdef = SphCaseDef.from_dict(case.case_def())
        init = case_particles(case)
        h = C.c_void_p()
        _check(L.sph_slab_group_create_axis(C.byref(self._cdef), C.byref(init.view), n,
                                            devices.ctypes.data_as(C.POINTER(C.c_int32)), int(axis),
                                            bounds.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(h)))
        self.axis = int(axis)
        self._h = h
        self.bounds = bounds
        self.members = []
        for i in range(n):
            m = C.c_void_p()
            _check(L.sph_slab_group_member(h, i, C.byref(m)))
            self.members.append(_SlabMember(self, m, case))
        for m in self.members:  # every slab runs the same motion program / body integration
            m._configure_bodies()

    def floatings(self) -> list:
        return self.members[0].floatings()

    def close(self) -> None:
        if getattr(self, "_h", None):
            for m in self.members:
                m.close()
            load_library().sph_slab_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def Run(self, nsteps: int) -> None:
        """nsteps whole steps on every slab (blocks until all slabs are done)."""
        _check(load_library().sph_slab_group_run(self._h, nsteps))

    run = Run

    def stats(self) -> list:
        return [m.stats() for m in self.members]

    def set_time(self, time: float, symplectic_dtpre: float = 0.0) -> None:
        """Restart time of every slab (JSph::InitRun with PartBegin)."""
        for m in self.members:
            m.set_time(time, symplectic_dtpre)

    def set_repartition(self, every: int, bound_weight: float = 0.3, tolerance: float = 0.05) -> None:
        """Re-balance the slabs' column bounds every `every` steps."""
        _check(load_library().sph_slab_group_set_repartition(self._h, every, bound_weight, tolerance))

    def set_overlap(self, on: bool) -> None:
        """Ghost exchange beside the interior items' interaction (default on), every slab."""
        _check(load_library().sph_slab_group_set_overlap(self._h, int(on)))

    def slab_info(self) -> list:
        return [m.slab_info() for m in self.members]

    def particles(self) -> dict:
        """Owned particles of all slabs, merged and sorted by idp."""
        parts = [m.particles() for m in self.members]
        cat = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
        o = np.argsort(cat["idp"], kind="stable")
        return {k: v[o] for k, v in cat.items()}


# ---- PART / case files (.bi4), SURVEY.md §8(f) row 2 ---------------------------------
def read_part(path: str) -> tuple[dict, dict]:
    """JPartDataBi4::LoadFilePart / LoadFileCase: (header values, particles by file order)."""
    L = load_library()
    h = SphPartHeader()
    _check(L.sph_part_read(os.fsencode(path), C.byref(h), None))
    hp = HostParticles(h.npok)
    hp.view.code = C.POINTER(C.c_uint16)()
    _check(L.sph_part_read(os.fsencode(path), C.byref(h), C.byref(hp.view)))
    p = hp.trimmed(h.npok)
    del p["code"]
    return h.as_dict(), p


def write_part(path: str, header: dict, particles: dict) -> None:
    """JPartDataBi4::AddPartInfo + AddPartData + SaveFilePart for host particle arrays."""
    h = SphPartHeader.from_dict(header)
    n = len(particles["idp"])
    h.npok = n
    hp = HostParticles(n, particles["idp"], particles["pos"], particles["vel"], particles["rhop"])
    _check(load_library().sph_part_write(os.fsencode(path), C.byref(h), C.byref(hp.view)))


def write_part_head(path: str, header: dict) -> None:
    """Part_Head.ibi4 (JPartDataHead) for a restart directory."""
    h = SphPartHeader.from_dict(header)
    _check(load_library().sph_part_head_write(os.fsencode(path), C.byref(h)))


def read_normals(path: str) -> np.ndarray:
    """<case>_Normals.nbi4 (JPartNormalData::LoadFile): PartNormals, double3[Nbound]."""
    L = load_library()
    n = C.c_uint32(0)
    _check(L.sph_normals_read(os.fsencode(path), 0, None, C.byref(n)))
    out = np.zeros((n.value, 3), np.float64)
    _check(L.sph_normals_read(os.fsencode(path), n.value, out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(n)))
    return out


def write_normals(path: str, normals: np.ndarray, dp: float, h: float, case_name: str = "") -> None:
    """<case>_Normals.nbi4 with the final normals of the boundary particles (as GenCase writes it)."""
    nor = np.ascontiguousarray(normals, np.float64).reshape(-1, 3)
    _check(load_library().sph_normals_write(os.fsencode(path), case_name.encode(), dp, h, 2.0 * h, len(nor),
                                            nor.ctypes.data_as(C.POINTER(C.c_double))))


def bi4_rewrite(src: str, dst: str) -> None:
    _check(load_library().sph_bi4_rewrite(os.fsencode(src), os.fsencode(dst)))


def part_header(case, stats: dict | None = None, cpart: int = 0, app_name: str = "dualsphysics_multilayer_amd",
                case_name: str = "CaseDambreak") -> dict:
    """PART header of a DamBreakCase (+ solver stats for time, counts, SymplecticDtPre)."""
    cd = case.case_def()
    k = case_derive(cd)
    pmin, pmax = case.pos.min(axis=0), case.pos.max(axis=0)
    st = stats or {}
    return dict(app_name=app_name, case_name=case_name, cpart=cpart, nout=int(st.get("nout", 0)),
                step=int(st.get("nstep", 0)), timestep=float(st.get("time", 0.0)),
                symplectic_dtpre=float(st.get("sym_dtpre", 0.0)) if case.step_algorithm == 2 else 0.0,
                domain_min=list(k["map_realposmin"]),
                domain_max=[k["map_realposmin"][i] + k["map_realsize"][i] for i in range(3)],
                case_np=case.np, case_nfixed=case.npb, case_nfluid=case.np - case.npb,
                dp=cd["dp"], h=cd["h"], b=cd["cteb"], rhop0=cd["rhop0"], gamma=cd["gamma"],
                massbound=cd["massbound"], massfluid=cd["massfluid"],
                map_posmin=list(cd["map_realposmin"]), map_posmax=list(cd["map_realposmax"]),
                case_posmin=pmin.tolist(), case_posmax=pmax.tolist(), pos_double=1,
                visco_type=1, visco=case.visco, viscoboundfactor=case.viscoboundfactor,
                gravity=list(case.gravity), mkbound=10, mkfluid=0,
                symmetry=int(bool(cd.get("symmetry", 0))))


def write_partfloat(path: str, floatings: list, parts: list, mkboundfirst: int = 10,
                    app: str = "dualsphysics_multilayer_amd") -> None:
    """PartFloat.fbi4 of a run: `floatings` = the case's bodies (XmlCase.floatings),
    `parts` = [{cpart, step, time, bodies: [SphGpuSingle.floatings() dicts]}]."""
    nft = len(floatings)
    u16 = lambda a: np.ascontiguousarray(a, np.uint16)  # noqa: E731
    u32 = lambda a: np.ascontiguousarray(a, np.uint32)  # noqa: E731
    f32 = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    head = [u16([f["mkbound"] for f in floatings]), u32([f["idbegin"] for f in floatings]),
            u32([f["count"] for f in floatings]), f32([f["massbody"] for f in floatings]),
            f32([f["masspart"] for f in floatings]), f32([f.get("radius", 0.0) for f in floatings])]
    cp = u32([p["cpart"] for p in parts])
    st = u32([p["step"] for p in parts])
    ts = np.ascontiguousarray([p["time"] for p in parts], np.float64)
    cen = np.ascontiguousarray([[b["center"] for b in p["bodies"]] for p in parts], np.float64).reshape(-1)
    arr = {k: f32([[b[k] for b in p["bodies"]] for p in parts]).reshape(-1)
           for k in ("fvel", "fomega", "facelin", "faceang")}
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    _check(load_library().sph_partfloat_write(path.encode(), app.encode(), mkboundfirst, nft,
                                              *[ptr(a) for a in head], len(parts), ptr(cp), ptr(st), ptr(ts),
                                              ptr(cen), *[ptr(arr[k]) for k in ("fvel", "fomega", "facelin",
                                                                                "faceang")]))


# ---- restart of floating bodies and mDBC (JSphCpu::InitFloating, JDsExtraData) -----------
def read_partfloat(path: str, cpart: int, nft: int) -> dict:
    """Body state of PART `cpart` in PartFloat.fbi4: center (nft, 3) f64, fvel / fomega f32, time."""
    center = np.zeros((nft, 3), np.float64)
    fvel = np.zeros((nft, 3), np.float32)
    fomega = np.zeros((nft, 3), np.float32)
    t = C.c_double()
    _check(load_library().sph_partfloat_read(path.encode(), int(cpart), int(nft), center.ctypes.data,
                                             fvel.ctypes.data, fomega.ctypes.data, C.byref(t)))
    return dict(center=center, fvel=fvel, fomega=fomega, time=t.value)


def read_extra_normals(path: str, casenbound: int, casenfloat: int) -> tuple[np.ndarray, bool]:
    """PartExtra_%04u.bi4: the normals by idp (vectors to the ghost node) and UseNormalsFt."""
    L = load_library()
    n, ft = C.c_uint32(), C.c_int32()
    _check(L.sph_extra_normals_read(path.encode(), casenbound, casenfloat, 0, None, C.byref(n), C.byref(ft)))
    out = np.zeros((n.value, 3), np.float32)
    _check(L.sph_extra_normals_read(path.encode(), casenbound, casenfloat, n.value, out.ctypes.data, C.byref(n),
                                    C.byref(ft)))
    return out, bool(ft.value)


def write_extra_normals(path: str, app: str, cpart: int, step: int, time: float, casenbound: int, casenfloat: int,
                        normals: np.ndarray, usenormalsft: bool) -> None:
    nor = np.ascontiguousarray(normals, np.float32).reshape(-1, 3)
    _check(load_library().sph_extra_normals_write(path.encode(), app.encode(), int(cpart), int(step), float(time),
                                                  int(casenbound), int(casenfloat), int(usenormalsft), len(nor),
                                                  nor.ctypes.data))
