#!/usr/bin/env python3
"""GPU check of one workload: compress on the device (compress_device), time
it, compare with the C restatement (cpu_ref, host threads) and report the BWT
routing (BZ2MI_BWT_STATS) and stage times.  Usage:
  rt_check.py <data> <MiB> [level] [p] [unit]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "bzip2-opencl_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bz2mi  # noqa: E402
from bz2mi import synth  # noqa: E402
from conftest import CpuRef  # noqa: E402

data, mib = sys.argv[1], int(sys.argv[2])
level = int(sys.argv[3]) if len(sys.argv) > 3 else 9
p = int(sys.argv[4]) if len(sys.argv) > 4 else 10
unit = int(sys.argv[5]) if len(sys.argv) > 5 else 10000
n = mib << 20
th = max(1, min(16, len(os.sched_getaffinity(0))))
t0 = time.time()
if data == "realtext":
    host = synth.realtext_bytes(n, threads=th)
elif data == "repeats":
    from test_gpu import _repeats
    host = _repeats(n)
elif data == "text":
    host = synth.text_bytes(n)
else:
    host = synth.random_bytes(n)
print(f"gen {time.time() - t0:.1f}s", flush=True)
dev = torch.device("cuda", 0)
x = torch.from_numpy(host).to(dev)
cap = bz2mi.compress_bound(n, level, unit)
out = torch.empty(cap, dtype=torch.uint8, device=dev)
ctx = bz2mi.Context(level, p, unit)
ctx.stats()
m = ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)
torch.cuda.synchronize()
os.environ.pop("BZ2MI_BWT_STATS", None)
ts = []
for _ in range(3):
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    m = ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t1)
tm = ctx.timings()
print(f"{data} {mib} MiB -{level} p={p} unit={unit}: {m} bytes ratio {m / n:.4f}, {min(ts) * 1e3:.2f} ms "
      f"= {n / min(ts) / 1e6:.0f} MB/s, stages {({k: round(v, 2) for k, v in tm.items()})}", flush=True)
got = out[:m].cpu().numpy().tobytes()
t0 = time.time()
want = CpuRef().compress(host.tobytes(), level, p, unit=unit, threads=th)
print(f"cpu_ref {time.time() - t0:.1f}s: equal = {got == want}", flush=True)
if got != want:
    a, b = np.frombuffer(got, np.uint8), np.frombuffer(want, np.uint8)
    k = min(len(a), len(b))
    d = np.nonzero(a[:k] != b[:k])[0]
    print("len", len(a), len(b), "first diff byte", d[0] if len(d) else k)
    sys.exit(1)
