"""Debug: bwt_text_kernel sums over one compression of C3 text (library built
with `make phases`; run with BZ2MI_LIBRARY=bzip2-opencl_amd/bz2mi/libbz2mi_ph.so)."""
import ctypes, os, sys
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(R, "bzip2-opencl_amd"))
import torch
import bz2mi
from bz2mi import synth

n = int(os.environ.get("MIB", "256")) << 20
kind = os.environ.get("DATA", "text")
if kind == "realtext":
    x = torch.from_numpy(synth.realtext_bytes(n, threads=8)).cuda()
elif kind == "repeats":
    sys.path.insert(0, os.path.join(R, "tests"))
    from test_gpu import _repeats
    x = torch.from_numpy(_repeats(n)).cuda()
else:
    x = torch.from_numpy(synth.text_bytes(n, synth.SEED_TEXT)).cuda()
ctx = bz2mi.Context(9, 10)
out = torch.empty(n + n // 8 + (1 << 20), dtype=torch.uint8, device="cuda")
ctx.compress_device(x.data_ptr(), n, out.data_ptr(), out.numel())
torch.cuda.synchronize()
L = bz2mi.lib()
buf = (ctypes.c_ulonglong * 16)()
print("rc", L.bz2mi_debug_phases(4, buf))
v = list(buf)
nb = max(1, v[8])
print(f"blocks {v[8]}  per block: total {v[9] / nb / 100:.1f} us, setup {v[0] / nb / 100:.1f}, sort {v[1] / nb / 100:.1f}, "
      f"copy {v[2] / nb / 100:.1f}, resolve {v[14] / nb / 100:.1f}, slowest block {v[15] / 100:.1f};  "
      f"flagged {v[11] / nb:.1f}, rounds {v[3] / nb:.1f}")
print(f"  sorts {v[4] / nb:.1f} ({v[7] / nb:.0f} elems, tie rounds {v[10] / nb:.1f}), partitions {v[5] / nb:.1f} "
      f"({v[6] / nb:.0f} elems)")
print(f"  wave-busy per block: sorts {v[12] / nb / 100:.1f} us, partitions {v[13] / nb / 100:.1f} us "
      f"(/16 = {(v[12] + v[13]) / nb / 1600:.1f} us of the sort phase)")
print("rc", L.bz2mi_debug_phases(5, buf))
r = list(buf)
nr = max(1, r[8])
print(f"  deferred: {r[8]} blocks with deferred groups, {r[2] / nr:.0f} groups per such block (max {r[9]}); "
      f"sent back: group>64 {r[10]}, periodic {r[11]}, no progress {r[12]}, pair list {r[13]}, work queue {r[14]}, "
      f"partition depth {r[15]}")
print(f"  resolve work per deferring block: rounds {r[3] / nr:.1f}, jump iterations {r[4] / nr:.1f}, plain-comparison "
      f"passes {r[7]} in all")
print(f"  resolve time per deferring block (thread 0): isa/marks {r[0] / nr / 100:.1f} us, pairs+groups "
      f"{r[1] / nr / 100:.1f}, links {r[5] / nr / 100:.1f}, step 3 + count (rounds before the last) {r[6] / nr / 100:.1f}")
print("rc", L.bz2mi_debug_phases(7, buf))
x = list(buf)
print(f"  wave time per block: tie rounds {x[0] / nb / 100:.1f} us, tied pairs {x[1] / nb / 100:.1f} us")
print(f"  walks: plain comparisons {x[2]} steps in all (longest {x[3]}), deferred comparisons {x[4]} steps (longest "
      f"{x[5]}); slowest resolve {x[6] / 100:.1f} us, slowest sort phase {x[7] / 100:.1f} us")
print(f"  setup to (thread 0, cumulative per block): text+mask {x[8] / nb / 100:.1f} us, pair counts {x[9] / nb / 100:.1f}, "
      f"starts+order {x[10] / nb / 100:.1f}, pair list {x[11] / nb / 100:.1f}, scatter = setup total")
print("timings", ctx.timings())
