"""Builds the HIP core libsphcore.so for gfx950, in-tree (no JIT cache).

Each translation unit is compiled separately (parallel) and linked with hipcc.
The product library never links the oracle.

One diagnostic define exists, for fast kernel A/B builds only (`build(outdir=..., defines=
["SPH_DIAG_HEADLINE_ONLY"])`, profiles/ab.sh): it compiles just the interaction kernels of the
BASELINE headline workloads (cfg2's k_fluid_tiled<10,false,1>, cfg5's k_nn_tiled<2,3,*>) and
makes every other case throw.  The product build never sets it.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUTDIR = os.path.join(HERE, "lib")
LIBNAME = "libsphcore.so"
SOURCES = ["sph_divide.hip", "sph_interaction.hip", "sph_interaction_tiled.hip", "sph_nn.hip", "sph_ext.hip", "sph_step.hip", "sph_slab.hip", "sph_mdbc.hip", "sph_bodies.hip",
           "sph_solver.cpp", "sph_comm.cpp", "sph_bi4.cpp", "sph_capi.cpp"]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
LDFLAGS = ["-L" + os.path.join(ROCM, "lib"), "-lrccl", "-Wl,-rpath," + os.path.join(ROCM, "lib"), "-pthread"]
ARCH = os.environ.get("SPH_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the HIP core cannot be built")


CXXFLAGS = [
    "-O3",
    "-std=c++17",
    "-fPIC",
    "--offload-arch=" + ARCH,
    "-ffp-contract=fast",
    "-munsafe-fp-atomics",
    "-fno-slp-vectorize",  # packed-f32 SLP adds v_mov shuffles in the pair loops (guide §B)
    "-Wall",
    "-Wno-unused-function",
]


def lib_path() -> str:
    return os.path.join(OUTDIR, LIBNAME)


def _deps(obj: str, src: str) -> list:
    """The headers a translation unit included (its -MMD file), or every header if unknown."""
    dfile = obj + ".d"
    if os.path.exists(dfile):
        text = open(dfile).read().replace("\\\n", " ")
        files = text.split(":", 1)[1].split() if ":" in text else []
        if files and all(os.path.exists(f) for f in files):
            return [src] + files
    deps = [src] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith((".hpp", ".h"))]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "sphcore.h"))
    return deps


def _stale(obj: str, src: str) -> bool:
    if not os.path.exists(obj):
        return True
    return os.path.getmtime(obj) < max(os.path.getmtime(d) for d in _deps(obj, src))


def build(force: bool = False, verbose: bool = False, outdir: str | None = None, defines: list | None = None) -> str:
    """Build libsphcore.so; `outdir`/`defines` make diagnostic variants (e.g. ablations)."""
    global OUTDIR
    saved = OUTDIR
    if outdir:
        OUTDIR = outdir
    try:
        return _build(force, verbose, defines or [])
    finally:
        OUTDIR = saved


def _build(force: bool, verbose: bool, defines: list) -> str:
    os.makedirs(os.path.join(OUTDIR, "obj"), exist_ok=True)
    cc = hipcc()
    objs = []
    jobs = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OUTDIR, "obj", s + ".o")
        objs.append(obj)
        if force or defines or _stale(obj, src):
            lang = ["-x", "hip"] if s.endswith(".hip") else []
            jobs.append([cc] + CXXFLAGS + ["-D" + d for d in defines] + lang +
                        ["-MMD", "-MF", obj + ".d", "-c", src, "-o", obj])
    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
            for cmd, r in zip(jobs, ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs)):
                if verbose or r.returncode:
                    sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
                if r.returncode:
                    raise RuntimeError("HIP compile failed: %s" % cmd[-3])
    out = lib_path()
    if jobs or not os.path.exists(out):
        # linked beside and renamed into place: a reader (a running test, a copy of the tree)
        # sees the old library or the new one, never a half-written file
        tmp = out + ".tmp%d" % os.getpid()
        cmd = [cc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs + LDFLAGS
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
        os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose="-v" in sys.argv))
