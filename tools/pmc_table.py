"""Summarise tools/pmc.sh output: per kernel, the counters summed over the
dispatches of the timed step (the last dispatch of each kernel)."""
import csv, glob, os, sys, collections
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = collections.defaultdict(dict)
for f in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    last = {}
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("bz2mi::", "")
        last.setdefault(k, {})
        d = int(r["Dispatch_Id"])
        last[k].setdefault(d, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    for k, ds in last.items():
        d = max(ds)
        vals[k].update(ds[d])
names = sorted({c for v in vals.values() for c in v})
w = csv.writer(sys.stdout)
w.writerow(["kernel"] + names)
for k in sorted(vals):
    w.writerow([k] + ["%.4g" % vals[k].get(c, float("nan")) for c in names])
