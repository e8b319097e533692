"""Summarise a rocprofv3 kernel + memory-copy trace of profiles/slab_overlap.py.

    python3 profiles/overlap_summary.py <rocprof dir> <out.json>

Per launching host thread (= one slab of the in-process group): the ghost-record copies
(device-to-device, the exchange after the divide) and that slab's interior k_fluid_tiled
launches (grid of nblocks - 64 blocks; the face launch uses the full grid), and how much of
each copy's interval lies inside an interior launch of the same slab.  Also the per-kernel
time of the exchange kernels per divide (k_pack_*, k_face_*, k_ghost_*, k_unpack*).
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
    return n[5:] if n.startswith("void ") else n


def main(src, dst):
    ks = rows(src, "kernel_trace.csv")
    ms = rows(src, "memory_copy_trace.csv")
    if not ks:
        raise SystemExit("no kernel trace under " + src)
    grid_key = next(k for k in ("Grid_Size_X", "Grid_Size", "Grid_SizeX") if k in ks[0])
    wg_key = next(k for k in ("Workgroup_Size_X", "Workgroup_Size", "Workgroup_SizeX") if k in ks[0])
    tid = "Thread_Id"
    interior = collections.defaultdict(list)
    face = collections.defaultdict(list)
    exch = collections.defaultdict(lambda: [0, 0.0])
    for r in ks:
        name = kname(r["Kernel_Name"])
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "k_fluid_tiled" in name:
            blocks = int(r[grid_key]) // max(1, int(r[wg_key]))
            (interior if blocks % 2048 else face)[r[tid]].append((t0, t1))
        for pre in ("k_pack_", "k_face_", "k_ghost_", "k_unpack"):
            if name.startswith(pre):
                exch[name][0] += 1
                exch[name][1] += (t1 - t0) * 1e-3
    copies = [r for r in ms if "DEVICE_TO_DEVICE" in r.get("Direction", r.get("Kind", "")).upper()
              or r.get("Source_Agent_Id") == r.get("Destination_Agent_Id")]
    per = collections.defaultdict(lambda: {"copies": 0, "copy_us": 0.0, "overlapped_us": 0.0, "copies_inside": 0})
    for r in copies:
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        p = per[r.get(tid, "?")]
        p["copies"] += 1
        p["copy_us"] += (t1 - t0) * 1e-3
        ov = 0
        for a, b in interior.get(r.get(tid, "?"), []):
            ov += max(0, min(t1, b) - max(t0, a))
        p["overlapped_us"] += ov * 1e-3
        p["copies_inside"] += 1 if ov > 0 else 0
    tot = {k: sum(p[k] for p in per.values()) for k in ("copies", "copy_us", "overlapped_us", "copies_inside")}
    out = {
        "slabs_seen": len(per),
        "interior_launches": sum(len(v) for v in interior.values()),
        "face_launches": sum(len(v) for v in face.values()),
        "interior_ms_avg": (sum((b - a) for v in interior.values() for a, b in v) * 1e-6 /
                            max(1, sum(len(v) for v in interior.values()))),
        "face_ms_avg": (sum((b - a) for v in face.values() for a, b in v) * 1e-6 /
                        max(1, sum(len(v) for v in face.values()))),
        "d2d_copies": tot,
        "fraction_of_copy_time_inside_an_interior_launch": tot["overlapped_us"] / max(tot["copy_us"], 1e-9),
        "per_slab_thread": dict(per),
        "exchange_kernels_us_total": {k: {"calls": v[0], "us": v[1], "avg_us": v[1] / max(1, v[0])}
                                      for k, v in sorted(exch.items())},
    }
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "per_slab_thread"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
