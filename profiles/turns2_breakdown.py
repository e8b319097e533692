"""Per-slab kernel breakdown of a full-step turns run (SPH_SLAB_TURNS=2) from its
rocprofv3 kernel trace: for every slab (host thread) the kernels of the timed steps (from
the slab's 3rd interaction launch on), summed per kind and divided by the interaction calls.

    python3 profiles/turns2_breakdown.py <run_kernel_trace.csv> [out.json]
"""
import collections
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
by_thr = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sphx::", "")
    base = name.split("<")[0]
    by_thr[r["Thread_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), base, int(r["Grid_Size_X"])))
# GPU-idle intervals of the whole timeline (no kernel of any slab running), each attributed to
# the slab whose kernel starts right after it: "own" when the kernel that ended right before it
# is of the same slab (its launch gaps, its host wait per divide), "handover" when another
# slab's (the turn chain of the measurement mode: slab r's turn starts after slab r-1's ends)
allk = sorted((s, e, thr) for thr, ev in by_thr.items() for (s, e, _, _) in ev)
idle_own = collections.defaultdict(float)
idle_hand = collections.defaultdict(float)
tstart = {}
busy_end, last_thr = None, None
for s, e, thr in allk:
    if busy_end is not None and s > busy_end:
        (idle_own if thr == last_thr else idle_hand)[(thr, s)] = (s - busy_end) / 1e3
    if busy_end is None or e >= busy_end:
        busy_end, last_thr = e, thr
res = {}
for thr, ev in by_thr.items():
    ev.sort()
    inter = [i for i, e in enumerate(ev) if e[2].startswith("k_fluid_tiled")]
    if len(inter) < 4:
        continue
    t0 = ev[inter[2]][0]  # skip the first two interactions (the warm-up)
    sel = [e for e in ev if e[0] >= t0]
    ncalls = sum(1 for e in sel if e[2].startswith("k_fluid_tiled"))
    acc = collections.defaultdict(float)
    for s, e, n, _ in sel:
        acc[n] += (e - s) / 1e3  # us
    own = sum(v for (t, s0), v in idle_own.items() if t == thr and s0 >= t0)
    hand = sum(v for (t, s0), v in idle_hand.items() if t == thr and s0 >= t0)
    res[thr] = {"interaction_calls": ncalls,
                "us_per_call": {k: round(v / ncalls, 2) for k, v in sorted(acc.items(), key=lambda kv: -kv[1])},
                "total_us_per_call": round(sum(acc.values()) / ncalls, 1),
                "idle_own_us_per_call": round(own / ncalls, 1),
                "idle_handover_us_per_call": round(hand / ncalls, 1)}
out = {"note": "cfg3 8-slab split, SPH_SLAB_TURNS=2 (each slab's kernels alone on the GPU), in-place ghosts; "
               "per slab (host thread): kernel time per interaction call (two calls per Symplectic step), "
               "from the slab's 3rd interaction on; GPU-idle time before the slab's kernels, after a kernel "
               "of its own (idle_own: launch gaps, host waits) or of another slab (idle_handover: the "
               "measurement mode's turn chain)", "slabs": res}
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
for thr, v in res.items():
    top = list(v["us_per_call"].items())[:9]
    print(thr, v["interaction_calls"], v["total_us_per_call"], v["idle_own_us_per_call"],
          v["idle_handover_us_per_call"], top)
