"""Summarise rocprofv3 --pmc passes: mean counter value per kernel (per dispatch)."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
res = collections.defaultdict(dict)
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in acc.items():
        res[k][c] = sum(v) / len(v)
if len(sys.argv) > 2:
    json.dump(res, open(sys.argv[2], "w"), indent=1, sort_keys=True)
for k in sorted(res):
    print(k)
    for c in sorted(res[k]):
        print("   %-28s %.4g" % (c, res[k][c]))
