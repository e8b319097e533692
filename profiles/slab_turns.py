"""One slab's own step on one GPU, the other slabs kept out of its window.

    SPH_SLAB_TURNS=1|2 python3 profiles/slab_turns.py [--slabs 8] [--steps 10] [--repeat 2]
    (under rocprofv3 --kernel-trace for the committed trace: --repeat 1 --only 1)

BASELINE cfg3 (the 10M Symplectic + DDT1 dam break) in its 8-slab split, in-process on one
MI355X, in the turns measurement mode of the in-process transport (SPH_SLAB_TURNS=1): slab
r's interaction — its interior items, the transfer and scatter of its ghost records on its
exchange stream, its face items — starts on the GPU only after slab r-1's interaction of
the same step has ended, and likewise the kernels of its divide after the exchange.  So each
slab's interaction and divide run with no other slab's interaction or divide beside them,
as each rank's do on its own GPU; the slabs' exchanges (pack, face counts, migrants) and
updates still run side by side.  SPH_SLAB_TURNS=2 chains the update kernels and the
exchange's pack kernels too (every kernel of a slab's step alone on the GPU, except the
few-us face-message and migrant copies and the unpack): the per-slab phase times are then
uncontended by the other slabs.  The transfers are device-to-device copies (blit kernels in
the block slots the interior launch leaves free); on the 8-GPU node they are RCCL
send/receive over one xGMI link per face.

Per slab and step, from its own streams' HIP events (sph_solver_timing): the interaction
window per call (interior + ghost transfer + scatter + face items) and the divide kernels per
call, in three modes, alternating repeats:
  overlap      the ghost records in flight beside the interior items (rows cut at the face
               columns: an interior list, then a face list of one-column items);
  inplace_cut  the ghosts in place before the interaction, the same cut items (SPH_SLAB_CUT=1);
  inplace      the ghosts in place, rows not cut (full items: the default).
Prints one JSON line per run and a final summary.
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
from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition  # noqa: E402


MODES = {"overlap": (1, 1), "inplace_cut": (0, 1), "inplace": (0, 0)}  # (overlap, cut)


def run(case, bounds, mode, steps, warmup, axis=0):
    overlap, cut = MODES[mode]
    os.environ["SPH_SLAB_CUT"] = str(cut)
    g = SphSlabGroup(case, np.asarray(bounds, np.int32), axis=axis)
    os.environ.pop("SPH_SLAB_CUT")
    g.set_overlap(bool(overlap))
    g.run(warmup)  # a group run returns with every slab synchronised
    for m in g.members:
        m.set_timing(True)
    t0 = time.perf_counter()
    g.run(steps)
    wall = 1e3 * (time.perf_counter() - t0) / steps
    ph = []
    for m in g.members:
        p, n = m.timing()
        ph.append({"interaction": round(float(p[0]), 4), "update": round(float(p[1]), 4),
                   "divide": round(float(p[2]), 4)})
    own = [int(m.stats()["np"]) for m in g.members]
    g.close()
    return {"mode": mode, "wall_ms_per_step": round(wall, 3), "owned_np": own, "phases_ms_per_call": ph}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slabs", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--only", choices=tuple(MODES), default=None, help="one mode only (e.g. under rocprofv3)")
    ap.add_argument("--modes", default=None, help="comma-separated subset of the modes")
    ap.add_argument("--dp", type=float, default=0.00205)
    ap.add_argument("--bound-weight", type=float, default=None, help="slab_partition's bound weight (default 0.3)")
    ap.add_argument("--axis", type=int, default=0, choices=(0, 1), help="slab axis: 0 x-slabs, 1 y-slabs")
    a = ap.parse_args()
    if os.environ.get("SPH_SLAB_TURNS") not in ("1", "2"):
        raise SystemExit("run with SPH_SLAB_TURNS=1 or 2 (the turns measurement modes)")
    case = DamBreakCase(a.dp, step_algorithm=2, tdensity=1)
    bw = 0.3 if a.bound_weight is None else a.bound_weight
    bounds = [int(x) for x in slab_partition(case, a.slabs, bw, a.axis)]
    res = {"workload": "cfg3", "np": int(case.np), "axis": a.axis, "bounds": bounds, "steps": a.steps,
           "turns_mode": int(os.environ["SPH_SLAB_TURNS"]), "bound_weight": a.bound_weight, "runs": []}
    modes = [a.only] if a.only is not None else (a.modes.split(",") if a.modes else list(MODES))
    for _ in range(a.repeat):
        for ov in modes:
            r = run(case, bounds, ov, a.steps, a.warmup, a.axis)
            res["runs"].append(r)
            print("progress", json.dumps(r), flush=True)
    summ = {}
    for ov in modes:
        rs = [r for r in res["runs"] if r["mode"] == ov]
        n = len(rs[0]["phases_ms_per_call"])
        best = lambda k, i: min(r["phases_ms_per_call"][i][k] for r in rs)  # noqa: E731
        summ[ov] = {
            "interaction_ms": [best("interaction", i) for i in range(n)],
            "divide_ms": [best("divide", i) for i in range(n)],
            "update_ms": [best("update", i) for i in range(n)],
            "wall_ms_per_step": min(r["wall_ms_per_step"] for r in rs),
        }
        # a slab's own step (Symplectic: two interactions, updates and divides per step)
        summ[ov]["slab_kernels_ms_per_step"] = [
            round(2 * (summ[ov]["interaction_ms"][i] + summ[ov]["update_ms"][i] + summ[ov]["divide_ms"][i]), 4)
            for i in range(n)]
    res["summary_min_over_repeats"] = summ
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
