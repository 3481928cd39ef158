"""Debug: bwt_finish (prefix doubling, repeat pairs) sums over one compression
(library built with `make variant VAR=ph`; run with
BZ2MI_LIBRARY=bzip2-opencl_amd/bz2mi/libbz2mi_ph.so).  DATA realtext|text|random,
UNIT 10000|100000, MIB."""
import ctypes, os, sys
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(R, "bzip2-opencl_amd"))
import torch
import bz2mi
from bz2mi import synth

n = int(os.environ.get("MIB", "256")) << 20
kind = os.environ.get("DATA", "realtext")
unit = int(os.environ.get("UNIT", "100000"))
if kind == "realtext":
    x = torch.from_numpy(synth.realtext_bytes(n, threads=8)).cuda()
elif kind == "repeats":
    x = torch.from_numpy(synth.repeats_bytes(n)).cuda()
elif kind == "random":
    x = torch.from_numpy(synth.random_bytes(n)).cuda()
else:
    x = torch.from_numpy(synth.text_bytes(n, synth.SEED_TEXT)).cuda()
ctx = bz2mi.Context(9, 10, unit)
out = torch.empty(n + n // 8 + (1 << 20), dtype=torch.uint8, device="cuda")
ctx.compress_device(x.data_ptr(), n, out.data_ptr(), out.numel())
torch.cuda.synchronize()
L = bz2mi.lib()
buf = (ctypes.c_ulonglong * 16)()
print("rc", L.bz2mi_debug_phases(6, buf))
v = list(buf)
nb = max(1, v[0])
print(f"{kind} unit {unit}: {v[0]} blocks doubled; per block: {v[3] / nb:.0f} groups (max {v[10]}), "
      f"total {v[1] / nb / 100:.1f} us (slowest {v[2] / 100:.1f}), labels {v[12] / nb / 100:.1f}, "
      f"pair passes {v[11] / nb / 100:.1f}; rounds {v[4] / nb:.1f} (max {v[5]})")
print(f"  first pair pass: decided {v[6] / nb:.0f}, undecided pairs {v[7] / nb:.0f}, groups left {v[8] / nb:.0f}")
print("timings", ctx.timings())
