"""Summarise tools/pmc.sh output: one row per dispatch of the bz2mi kernels
(in dispatch order), every counter of every pass."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_random"
only = sys.argv[2] if len(sys.argv) > 2 else ""
rows = collections.defaultdict(dict)  # (pass-local dispatch order, kernel) -> counters
for f in sorted(glob.glob(os.path.join(root, "*", "*counter_collection.csv"))):
    per = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("bz2mi::", "")
        if "bz2mi" not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        names[d] = k
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for j, d in enumerate(sorted(per)):
        rows[(j, names[d])].update(per[d])
cols = sorted({c for v in rows.values() for c in v})
w = csv.writer(sys.stdout)
w.writerow(["#", "kernel"] + cols)
for (j, k), v in sorted(rows.items()):
    if only and only not in k:
        continue
    w.writerow([j, k] + ["%.4g" % v.get(c, float("nan")) for c in cols])
