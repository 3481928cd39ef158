"""Host-side timeline of one unit-protocol step at N=1 (4 units of 256 MiB):
wall time when each call of bz2mi.shard's protocol returns."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bzip2-opencl_amd"))
import torch
import bz2mi
from bz2mi import shard

K, U = 4, 256 << 20
dev = torch.device("cuda", 0)
g = torch.Generator(device="cuda").manual_seed(0x5EED0001)
x = torch.randint(0, 256, (K * U,), dtype=torch.uint8, device="cuda", generator=g)
H = bz2mi.unit_halo(9, 10000)
ctx = bz2mi.Context(9, 10)
units = {i: shard.DeviceUnit(ctx, dev) for i in range(K)}
owners = [0] * K
T0 = [0.0]
log = []


def wrap(u, name, i):
    f = getattr(u, name)

    def w(*a):
        r = f(*a)
        log.append((time.perf_counter() - T0[0], name, i))
        return r
    setattr(u, name, w)


for i, u in units.items():
    for m in ("chain", "sums", "encode", "assemble"):
        wrap(u, m, i)
for step in range(3):
    torch.cuda.synchronize()
    log.clear()
    T0[0] = time.perf_counter()
    for i in range(K):
        lo = i * U
        hi = min(K * U, lo + U + H)
        units[i].begin(x[lo:hi], U, hi - lo - U, hi == K * U)
    log.append((time.perf_counter() - T0[0], "begin all", -1))
    lay = shard.compress_units(units, owners, 10, 9)
    torch.cuda.synchronize()
    log.append((time.perf_counter() - T0[0], "done", -1))
for t, n, i in log:
    print(f"{t * 1e3:8.3f} ms  {n} {i}")
