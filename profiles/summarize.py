"""Summarise one profiles/collect.sh run into <dst>/kernel_stats.csv + pmc_traffic.json.

HBM traffic per launch (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are in KiB
per dispatch; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read
(16 B/lane), so traffic = 2 * FETCH_SIZE + WRITE_SIZE.  The dominant kernels' loads
are 16-B-per-lane float4 streams (poscell, velrhop); the 4-B press loads are
uncalibrated, so the figure is an estimate at that accuracy.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def kname(n):
    n = n.split("(")[0]
    return n[5:] if n.startswith("void ") else n


def counters(root):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[(kname(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
    avg_ns = {}
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            avg_ns[kname(r["Name"])] = float(r["AverageNs"])
    fetch, write = counters(os.path.join(src, "fetch")), counters(os.path.join(src, "write"))
    out = {}
    for (k, c), (v, n) in fetch.items():
        if c != "FETCH_SIZE":
            continue
        w = write.get((k, "WRITE_SIZE"), (0.0, 0))[0]
        out[k] = {
            "FETCH_SIZE_KiB": v,
            "WRITE_SIZE_KiB": w,
            "dispatches": n,
            "traffic_bytes_per_launch": (2.0 * v + w) * 1024.0,
            "avg_ns": avg_ns.get(k),
        }
    json.dump(out, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1, sort_keys=True)
    for k in sorted(out, key=lambda k: -(out[k]["avg_ns"] or 0)):
        o = out[k]
        print("%-40s %10.1f us  traffic %8.2f MB/launch" % (k[:40], (o["avg_ns"] or 0) / 1e3,
                                                            o["traffic_bytes_per_launch"] / 1e6))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
