"""Print a rocprofv3 kernel_stats.csv as a short table (ms per call)."""
import csv
import sys

for path in sys.argv[1:]:
    print(path)
    for r in csv.DictReader(open(path)):
        name = r["Name"].split("(")[0].replace("bz2mi::", "")[:36]
        print(f"  {name:36s} {r['Calls']:>4s} {float(r['AverageNs']) / 1e6:9.3f} ms {float(r['Percentage']):6.2f}%")
