"""Summarise a rocprofv3 kernel + memory-copy trace of profiles/slab_turns.py (turns mode).

    python3 profiles/turns_summary.py <rocprof dir> <out.json> [timeline.txt]

Per slab (the host thread that launches its kernels): its interior k_fluid_tiled launches
(grid of nblocks - 64 blocks, solver stream), the ghost-record copies of the same slab
(blit kernels __amd_rocclr_copyBuffer or DMA copies, on its exchange stream) and its
k_ghost_scatter; whether each copy / scatter STARTS inside the same slab's interior launch;
and, as the isolation check of the turns mode, how much of each interior launch another
slab's k_fluid_tiled overlaps.  Optionally a text timeline of one step of one slab.
"""
import collections
import csv
import glob
import json
import os
import sys


def rows(root, suffix):
    out = []
    for f in glob.glob(os.path.join(root, "**", "*" + suffix), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def kname(n):
    n = n.split("(")[0].split("<")[0]
    n = n[5:] if n.startswith("void ") else n
    return n.split("::")[-1]


def main(src, dst, timeline=None):
    ks = rows(src, "kernel_trace.csv")
    if not ks:
        raise SystemExit("no kernel trace under " + src)
    mc = rows(src, "memory_copy_trace.csv")
    by = collections.defaultdict(list)  # thread -> [(t0, t1, name, stream, blocks)]
    for r in ks:
        blocks = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        by[r["Thread_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kname(r["Kernel_Name"]),
                                   r["Stream_Id"], blocks))
    for r in mc:
        if "DEVICE_TO_DEVICE" in r.get("Direction", ""):
            by[r["Thread_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "dma_copy_d2d",
                                       r["Stream_Id"], 0))
    interior_all = []  # (thread, t0, t1)
    for th, ev in by.items():
        for t0, t1, n, s, b in ev:
            if n.startswith("k_fluid_tiled") and b % 2048:
                interior_all.append((th, t0, t1))
    per = {}
    for th, ev in by.items():
        ev.sort()
        inter = [(t0, t1, s) for t0, t1, n, s, b in ev if n.startswith("k_fluid_tiled") and b % 2048]
        if not inter:
            continue
        istreams = {s for _, _, s in inter}
        copies = [(t0, t1) for t0, t1, n, s, b in ev
                  if n in ("__amd_rocclr_copyBuffer", "dma_copy_d2d") and s not in istreams]
        scat = [(t0, t1) for t0, t1, n, s, b in ev if n == "k_ghost_scatter" and s not in istreams]
        face = [(t0, t1) for t0, t1, n, s, b in ev if n.startswith("k_fluid_tiled") and not b % 2048]

        def inside(lst):
            return sum(1 for t0, _ in lst if any(a <= t0 < b for a, b, _ in inter))

        other = 0
        tot = 0
        for a, b, _ in inter:
            tot += b - a
            for th2, c, d in interior_all:
                if th2 != th:
                    other += max(0, min(b, d) - max(a, c))
        per[th] = {
            "interior_launches": len(inter),
            "interior_us_avg": sum(b - a for a, b, _ in inter) * 1e-3 / len(inter),
            "ghost_copies": len(copies), "ghost_copies_starting_inside_own_interior": inside(copies),
            "ghost_copy_us_avg": sum(b - a for a, b in copies) * 1e-3 / max(1, len(copies)),
            "scatters": len(scat), "scatters_starting_inside_own_interior": inside(scat),
            "face_launches": len(face), "face_us_avg": sum(b - a for a, b in face) * 1e-3 / max(1, len(face)),
            "other_slabs_interior_overlap_fraction": other / max(tot, 1),
        }
    out = {"slabs": per,
           "all_copies_inside": sum(v["ghost_copies_starting_inside_own_interior"] for v in per.values()),
           "all_copies": sum(v["ghost_copies"] for v in per.values()),
           "all_scatters_inside": sum(v["scatters_starting_inside_own_interior"] for v in per.values()),
           "all_scatters": sum(v["scatters"] for v in per.values())}
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))
    if timeline:
        # one interior launch of a slab with two faces (the busiest thread), +-0.5 ms around it
        th = max(per, key=lambda t: (per[t]["ghost_copies"] > 0, per[t]["interior_us_avg"]))
        ev = sorted(by[th])
        inter = [(t0, t1) for t0, t1, n, s, b in ev if n.startswith("k_fluid_tiled") and b % 2048]
        a, b = inter[len(inter) // 2]
        t00 = a - 500_000
        with open(timeline, "w") as f:
            f.write("thread %s, one interior launch (times in us from 0.5 ms before it)\n" % th)
            for t0, t1, n, s, bl in ev:
                if t1 >= t00 and t0 <= b + 500_000:
                    f.write("%10.1f %10.1f  stream %-4s %-28s blocks %d\n" % ((t0 - t00) * 1e-3, (t1 - t00) * 1e-3,
                                                                          s, n, bl))
        print("timeline ->", timeline)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
