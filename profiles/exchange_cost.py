"""Per-divide slab exchange cost from a rocprofv3 kernel trace of
`profiles/slab_cost.py --only eight` (BASELINE cfg3's 8-slab split in one process): the
exchange kernels' average duration per call and their sum per slab divide, beside the
interaction and divide kernels of the same run.  Usage: exchange_cost.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

EXCHANGE = ("k_pack_count", "k_pack_scan", "k_pack_write", "k_face_hdr", "k_face_scan", "k_unpack",
            "k_unpack_finish", "k_ghost_pack", "k_ghost_scatter", "k_fold", "k_small_sort")
DIVIDE = ("k_inc_classify", "k_inc_boxes", "k_inc_push", "k_items_place")


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("sphx::", "")
    return n.split("<")[0]


def main(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ndiv = len(d.get("k_inc_classify", [])) or 1  # one classify per slab divide
    print("slab divides in the trace: %d" % ndiv)
    tot = 0.0
    for k in EXCHANGE:
        if k in d:
            v = d[k]
            per = sum(v) / ndiv
            tot += per
            print("  %-18s calls %5d  avg %7.2f us  per divide %7.2f us" % (k, len(v), sum(v) / len(v), per))
    print("  exchange kernels per slab divide: %.1f us" % tot)
    for k in DIVIDE + ("k_fluid_tiled", "__amd_rocclr_copyBuffer"):
        if k in d:
            v = d[k]
            print("  %-24s calls %5d  avg %8.2f us" % (k, len(v), sum(v) / len(v)))


if __name__ == "__main__":
    main(sys.argv[1])
