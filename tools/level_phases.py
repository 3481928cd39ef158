"""Level-kernel phase sums (libbz2mi built with `make PHASES=1`): one
compression of MIB MiB of DATA; prints the wall-clock sums (us, thread 0 of
every workgroup, all level launches) of the partition phases."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bzip2-opencl_amd"))
import torch
import bz2mi

n = int(os.environ.get("MIB", "256")) << 20
from bz2mi import synth
x = torch.from_numpy(synth.text_bytes(n) if os.environ.get("DATA", "text") == "text" else synth.random_bytes(n)).cuda()
ctx = bz2mi.Context(9, 10)
out = torch.empty(n + n // 8 + (1 << 20), dtype=torch.uint8, device="cuda")
ctx.compress_device(x.data_ptr(), n, out.data_ptr(), out.numel())
torch.cuda.synchronize()
L = bz2mi.lib()
buf = (ctypes.c_ulonglong * 16)()
L.bz2mi_debug_phases(1, buf)
v = list(buf)
names = ["load+hist", "scan+scatter", "pack", "reserve", "push"]
print({names[k]: round(v[8 + k] / 100.0, 1) for k in range(5)}, "workgroups", v[14])
print("timings", ctx.timings())
