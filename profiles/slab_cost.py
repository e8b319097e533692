"""What the slab decomposition costs one rank, measured on one GPU (DESIGN.md §6 model).

    python3 profiles/slab_cost.py [--workload cfg3] [--steps 20] [--warmup 4]

Runs the same case and steps three ways and prints one JSON line:
  domain    one domain (SphGpuSingle): the single-GPU step;
  one_slab  the slab path with one rank (SphSlabGroup, bounds [0, ncx]): no neighbours, so
            no collective and no ghosts — the pure cost of the slab code path;
  faces     three in-process slabs [0, w) | [w, ncx - w) | [ncx - w, ncx) with w = 2W
            ghost columns (the narrowest slab allowed): the middle slab holds all but the two
            end strips and has BOTH faces, like an interior rank of the 8-GPU split, while its
            two neighbours are strips of a few thousand to a few hundred thousand particles
            whose concurrent work on the same GPU barely contends.  Its step minus the
            domain's step is the per-step cost of an interior rank's exchange: packs, the
            face-count round trip (one host wait per divide), migrants, ghost slots in the
            divide, the ghost pack, the ghost records' copies beside the interior items and
            the face items' launch after them.  The middle slab's interaction / divide /
            update phases come from its own stream's events.
The ghost records of a face travel here as device-to-device copies (LocalTransport); on
the 8-GPU node they cross one xGMI link (RCCL send/receive) beside the interior items.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from dualsphysics_multilayer_amd.case import DamBreakCase  # noqa: E402
from dualsphysics_multilayer_amd.core import SphGpuSingle, SphSlabGroup, slab_partition  # noqa: E402

# bench.py's workloads: cfg3 = the 10M Symplectic + DDT1 dam break, cfg2 = the 1M Verlet + DDT2 one
CFG = {"cfg3": dict(dp=0.00205, step_algorithm=2, tdensity=1), "cfg2": dict(dp=0.0045)}


def _sync(obj):
    if hasattr(obj, "sync"):
        obj.sync()


def timed(obj, steps, warmup, timing_of=None):
    """ms per step (wall, device synced; no timing events in that region) and, if asked,
    one member's phase times per step from a second run of the same length."""
    obj.run(warmup)
    _sync(obj)
    t0 = time.perf_counter()
    obj.run(steps)
    _sync(obj)
    ms = 1e3 * (time.perf_counter() - t0) / steps
    ph = None
    if timing_of is not None:
        timing_of.set_timing(True)
        obj.run(steps)
        _sync(obj)
        p, _ = timing_of.timing()  # ms per call of each phase: interaction, update, divide, mdbc
        ph = dict(zip(("interaction", "update", "divide", "mdbc"), (round(float(x), 4) for x in p)))
    return round(ms, 4), ph


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=tuple(CFG), default="cfg3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--repeat", type=int, default=2, help="alternating repeats of the three runs")
    ap.add_argument("--overlap", type=int, default=1, help="slab ghost overlap on (1) / off (0)")
    ap.add_argument("--only", choices=("domain", "one_slab", "faces", "left", "eight"), default=None,
                    help="one of the runs (e.g. under rocprofv3); left: [0, w) | [w, ncx), the big slab with one "
                         "face in the water, whose face launch runs after the strip's (a trace isolates it); "
                         "eight: BASELINE cfg3's 8-slab split in one process (its exchange kernels per divide "
                         "at the 8-GPU slab size, from a rocprofv3 trace)")
    a = ap.parse_args()
    case = DamBreakCase(**CFG[a.workload])
    ncx = int(slab_partition(case, 1)[-1])
    W = 1  # full cells, DBC: one ghost column per face
    w = 2 * W
    out = {"workload": a.workload, "np": int(case.np), "ncx": ncx, "steps": a.steps, "strip_columns": w,
           "overlap": a.overlap,
           "domain_ms": [], "one_slab_ms": [], "faces_ms": [], "domain_phases_ms": None, "faces_mid_phases_ms": None}
    for _ in range(a.repeat):
        if a.only in (None, "domain"):
            s = SphGpuSingle(case)
            ms, ph = timed(s, a.steps, a.warmup, s)
            s.close()
            out["domain_ms"].append(ms)
            out["domain_phases_ms"] = ph
        if a.only in (None, "one_slab"):
            g = SphSlabGroup(case, np.array([0, ncx], np.int32))
            ms, _ = timed(g, a.steps, a.warmup)
            g.close()
            out["one_slab_ms"].append(ms)
        if a.only in (None, "faces"):
            g = SphSlabGroup(case, np.array([0, w, ncx - w, ncx], np.int32))
            g.set_overlap(bool(a.overlap))
            ms, ph = timed(g, a.steps, a.warmup, g.members[1])
            out["faces_np"] = [int(m.stats()["np"]) for m in g.members]
            g.close()
            out["faces_ms"].append(ms)
            out["faces_mid_phases_ms"] = ph
        if a.only == "left":
            g = SphSlabGroup(case, np.array([0, w, ncx], np.int32))
            g.set_overlap(bool(a.overlap))
            ms, ph = timed(g, a.steps, a.warmup, g.members[1])
            out["left_np"] = [int(m.stats()["np"]) for m in g.members]
            g.close()
            out.setdefault("left_ms", []).append(ms)
            out["left_big_phases_ms"] = ph
        if a.only == "eight":
            g = SphSlabGroup(case, slab_partition(case, 8))
            g.set_overlap(bool(a.overlap))
            ms, ph = timed(g, a.steps, a.warmup, g.members[3])
            out["eight_np"] = [int(m.stats()["np"]) for m in g.members]
            g.close()
            out.setdefault("eight_ms", []).append(ms)
            out["eight_slab3_phases_ms"] = ph
        print("progress", json.dumps(out), flush=True)
    if a.only is None:
        d, o, f = min(out["domain_ms"]), min(out["one_slab_ms"]), min(out["faces_ms"])
        out["one_slab_over_domain"] = round(o / d, 4)
        out["faces_minus_domain_ms"] = round(f - d, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
