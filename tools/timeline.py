"""Kernel timeline summary of a rocprofv3 --kernel-trace run: the last step
(kernels after the last gap > 2 ms), per kernel name the summed duration, and
the union of kernel intervals (busy) against the step's span (idle = gaps
where no kernel runs)."""
import collections
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "bz2mi" in r["Kernel_Name"]]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("bz2mi::", ""))
            for r in rows)
# steps: split at gaps > 2 ms
steps, cur = [], [iv[0]]
for a in iv[1:]:
    if a[0] - max(x[1] for x in cur) > 2_000_000:
        steps.append(cur)
        cur = [a]
    else:
        cur.append(a)
steps.append(cur)
last = steps[-1]
t0, t1 = last[0][0], max(x[1] for x in last)
busy, end = 0, t0
for s, e, _ in last:
    if e <= end:
        continue
    busy += e - max(s, end)
    end = e
per = collections.defaultdict(lambda: [0, 0])
for s, e, n in last:
    per[n][0] += e - s
    per[n][1] += 1
print(f"steps found {len(steps)}; last step: span {(t1 - t0) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e6:.3f} ms, kernels {len(last)}")
for n, (d, c) in sorted(per.items(), key=lambda kv: -kv[1][0]):
    print(f"  {n[:48]:48s} {c:5d} x  {d / 1e6:8.3f} ms")
# the largest idle gaps with the kernels around them
gaps, end, prev = [], t0, None
for s, e, n in last:
    if s > end:
        gaps.append((s - end, prev, n))
    if e > end:
        end, prev = e, n
for g, a, b in sorted(gaps, reverse=True)[:8]:
    print(f"  gap {g / 1e3:8.1f} us after {a} before {b}")
