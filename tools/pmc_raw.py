"""Raw per-kernel sums of one rocprofv3 --pmc pass (counter_collection.csv):
python tools/pmc_raw.py <csv> [kernel-substring]  -> one JSON line per kernel
(counters summed over its dispatches, plus the dispatches' total ms)."""
import collections
import csv
import json
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
seen = collections.defaultdict(set)
flt = sys.argv[2] if len(sys.argv) > 2 else "bz2mi::"
for r in csv.DictReader(open(sys.argv[1])):
    if flt not in r["Kernel_Name"]:
        continue
    k = r["Kernel_Name"].split("(")[0].replace("bz2mi::", "").replace("void ", "")
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Dispatch_Id"] not in seen[k]:
        seen[k].add(r["Dispatch_Id"])
        acc[k]["_ms"] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-6
for k, c in sorted(acc.items()):
    print(json.dumps({"kernel": k, **{n: round(v, 3) for n, v in sorted(c.items())}}))
