"""Per-round doubling statistics of the 900 KB mode (BZ2MI_DBL_STATS) on
realtext: groups, large groups, pairs decided per round."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bzip2-opencl_amd"))
os.environ["BZ2MI_DBL_STATS"] = "1"
import torch
import bz2mi
from bz2mi import synth
n = int(os.environ.get("MIB", "256")) << 20
x = torch.from_numpy(synth.realtext_bytes(n, synth.SEED_REALTEXT, threads=8)).cuda()
ctx = bz2mi.Context(9, 10, 100000)
out = torch.empty(n + n // 4 + (1 << 20), dtype=torch.uint8, device="cuda")
ctx.compress_device(x.data_ptr(), n, out.data_ptr(), out.numel())
torch.cuda.synchronize()
print("timings", ctx.timings())
