"""Summarise a rocprofv3 kernel + memory-copy trace of profiles/slab_overlap.py.

    python3 profiles/overlap_summary.py <rocprof dir> <out.json>

The ghost-record copies on the slabs' exchange streams (DMA copies, or blit kernels) and
the interior k_fluid_tiled launches (grid of nblocks - 64 blocks; the face launches use the
full grid and run on the exchange streams): how much of the copy time passes while an
interior launch runs.  Also the per-kernel time of the exchange kernels (k_pack_*,
k_face_*, k_ghost_*, k_unpack*).
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


def main(src, dst):
    ks = rows(src, "kernel_trace.csv")
    if not ks:
        raise SystemExit("no kernel trace under " + src)
    # interior k_fluid_tiled launches (grid of nblocks - 64 blocks) and face launches (full
    # grid); the streams the face launches run on are the slabs' exchange streams, where
    # the ghost copies run (DMA copies of the memory-copy trace, or blit kernels)
    interior, face, xstreams = [], [], set()
    exch = collections.defaultdict(lambda: [0, 0.0])
    for r in ks:
        name = kname(r["Kernel_Name"])
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if name == "k_fluid_tiled":
            blocks = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
            if blocks % 2048:
                interior.append((t0, t1))
            else:
                face.append((t0, t1))
                xstreams.add(r["Stream_Id"])
        for pre in ("k_pack_", "k_face_", "k_ghost_", "k_unpack"):
            if name.startswith(pre):
                exch[name][0] += 1
                exch[name][1] += (t1 - t0) * 1e-3
    copies = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows(src, "memory_copy_trace.csv")
              if "DEVICE_TO_DEVICE" in r["Direction"] and r["Stream_Id"] in xstreams]
    copies += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks
               if kname(r["Kernel_Name"]) == "__amd_rocclr_copyBuffer" and r["Stream_Id"] in xstreams]
    cu = ov = 0
    inside = 0
    for t0, t1 in copies:
        cu += t1 - t0
        o = 0
        for a, b in interior:  # interior launches overlap each other only across slabs: clip
            o += max(0, min(t1, b) - max(t0, a))
        o = min(o, t1 - t0)
        ov += o
        inside += 1 if o > 0 else 0
    out = {
        "interior_launches": len(interior),
        "face_launches": len(face),
        "interior_ms_avg": sum(b - a for a, b in interior) * 1e-6 / max(1, len(interior)),
        "face_ms_avg": sum(b - a for a, b in face) * 1e-6 / max(1, len(face)),
        "ghost_copies": {"count": len(copies), "us": cu * 1e-3, "us_while_an_interior_launch_runs": ov * 1e-3,
                         "copies_overlapping_an_interior_launch": inside},
        "fraction_of_ghost_copy_time_while_an_interior_launch_runs": ov / max(cu, 1e-9),
        "exchange_kernels": {k: {"calls": v[0], "us": v[1], "avg_us": v[1] / max(1, v[0])}
                             for k, v in sorted(exch.items())},
    }
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
