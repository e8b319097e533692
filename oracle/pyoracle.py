"""ctypes binding of the CPU oracle (oracle/build/libsph_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from dualsphysics_multilayer_amd._abi import (
    HostParticles,
    SphCaseDef,
    SphConstants,
    SphInterOut,
    SphRunStats,
)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libsph_oracle.so")
# the same restatement without -ffast-math: the reference's own rounding-noise floor at
# the interaction level (fast-math vs strict IEEE of the same code, as SURVEY §8(c) measures
# it on whole runs)
LIB_STRICT = os.path.join(HERE, "build", "libsph_oracle_strict.so")


def build_oracle(force: bool = False, strict: bool = False) -> str:
    """Compile the oracle restatement with the reference's flags (Makefile_cpu:19-28), or
    (strict) the same without -ffast-math."""
    out = LIB_STRICT if strict else LIB
    src = os.path.join(HERE, "sph_oracle.cpp")
    hdr = os.path.join(HERE, "sph_oracle.h")
    abi = os.path.join(os.path.dirname(HERE), "include", "sphcore.h")  # the PODs it shares with the core
    if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(src), os.path.getmtime(hdr),
                                                                         os.path.getmtime(abi)):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["g++", "-O3", "-fopenmp"] + ([] if strict else ["-ffast-math"]) + ["-shared", "-fPIC", "-o", out, src]
    subprocess.check_call(cmd)
    return out


_libs = {}


def lib(strict: bool = False):
    if strict not in _libs:
        path = build_oracle(strict=strict)
        L = C.CDLL(path)
        vp = C.c_void_p
        L.or_last_error.restype = C.c_char_p
        L.or_case_derive.argtypes = [C.POINTER(SphCaseDef), C.POINTER(SphConstants)]
        L.or_create.argtypes = [C.POINTER(SphCaseDef), C.c_void_p, C.c_int, C.POINTER(vp)]
        L.or_destroy.argtypes = [vp]
        L.or_run.argtypes = [vp, C.c_uint32]
        L.or_stats.argtypes = [vp, C.POINTER(SphRunStats)]
        L.or_dt_trace.argtypes = [vp, C.POINTER(C.c_double), C.c_uint32, C.POINTER(C.c_uint32)]
        L.or_download.argtypes = [vp, C.c_void_p]
        L.or_interaction.argtypes = [vp, C.c_int, C.POINTER(SphInterOut)]
        L.or_count_pairs.argtypes = [vp, C.POINTER(C.c_uint64)]
        L.or_run_seconds.argtypes = [vp]
        L.or_run_seconds.restype = C.c_double
        L.or_threads.argtypes = [vp]
        _libs[strict] = L
    return _libs[strict]


def _check(r: int) -> None:
    if r != 0:
        raise RuntimeError("oracle error %d: %s" % (r, lib().or_last_error().decode()))


def derive(case_def: dict) -> dict:
    k = SphConstants()
    _check(lib().or_case_derive(C.byref(SphCaseDef.from_dict(case_def)), C.byref(k)))
    return k.as_dict()


class OracleSolver:
    """CPU restatement of JSphCpuSingle for the dam-break feature set."""

    def __init__(self, case, nthreads: int = 0, strict: bool = False):
        self.case = case
        self._L = lib(strict)
        self._cdef = SphCaseDef.from_dict(case.case_def())
        init = HostParticles(case.np, case.idp, case.pos, case.vel, case.rhop, boundnormal=getattr(case, "boundnormal", None))
        h = C.c_void_p()
        _check(self._L.or_create(C.byref(self._cdef), C.byref(init.view), nthreads, C.byref(h)))
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.or_destroy(self._h)
            self._h = None

    def run(self, nsteps: int) -> None:
        _check(self._L.or_run(self._h, nsteps))

    def stats(self) -> dict:
        s = SphRunStats()
        _check(self._L.or_stats(self._h, C.byref(s)))
        return s.as_dict()

    def dt_trace(self) -> np.ndarray:
        cnt = C.c_uint32()
        _check(self._L.or_dt_trace(self._h, None, 0, C.byref(cnt)))
        out = np.zeros(cnt.value, np.float64)
        _check(self._L.or_dt_trace(self._h, out.ctypes.data_as(C.POINTER(C.c_double)), cnt.value, C.byref(cnt)))
        return out

    def particles(self) -> dict:
        n = self.case.np
        hp = HostParticles(n)
        _check(self._L.or_download(self._h, C.byref(hp.view)))
        return hp.trimmed(hp.view.n)

    def interaction(self, interstep: int = 1) -> dict:
        n = self.stats()["np"]
        ar = np.zeros(n, np.float32)
        ace = np.zeros((n, 3), np.float32)
        out = SphInterOut(ar.ctypes.data_as(C.POINTER(C.c_float)), ace.ctypes.data_as(C.POINTER(C.c_float)), 0, 0, 0)
        _check(self._L.or_interaction(self._h, interstep, C.byref(out)))
        return dict(ar=ar, ace=ace, viscdtmax=out.viscdtmax, velmax=out.velmax, acemax=out.acemax)

    def count_pairs(self) -> np.ndarray:
        out = np.zeros(6, np.uint64)
        _check(self._L.or_count_pairs(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64))))
        return out

    def run_seconds(self) -> float:
        return self._L.or_run_seconds(self._h)

    def threads(self) -> int:
        return self._L.or_threads(self._h)
