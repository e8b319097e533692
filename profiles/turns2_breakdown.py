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
    res[thr] = {"interaction_calls": ncalls,
                "us_per_call": {k: round(v / ncalls, 2) for k, v in sorted(acc.items(), key=lambda kv: -kv[1])},
                "total_us_per_call": round(sum(acc.values()) / ncalls, 1)}
out = {"note": "cfg3 8-slab split, SPH_SLAB_TURNS=2 (each slab's kernels alone on the GPU), in-place ghosts; "
               "per slab (host thread): kernel time per interaction call (two calls per Symplectic step), "
               "from the slab's 3rd interaction on", "slabs": res}
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
for thr, v in res.items():
    top = list(v["us_per_call"].items())[:9]
    print(thr, v["interaction_calls"], v["total_us_per_call"], top)
