"""Phase stamps of one representative workgroup per kernel (libbz2mi built
with `make PHASES=1`): runs one compression of 256 MiB random bytes and prints
per-phase microseconds."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bzip2-opencl_amd"))
import torch
import bz2mi

n = int(os.environ.get("MIB", "256")) << 20
kind = os.environ.get("DATA", "random")
g = torch.Generator(device="cuda").manual_seed(0x5EED0001)
if kind == "random":
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
else:
    from bz2mi import synth
    gen = {"text": synth.text_bytes, "mixed": synth.mixed_bytes, "realtext": synth.realtext_bytes}[kind]
    x = torch.from_numpy(gen(n)).cuda()
ctx = bz2mi.Context(9, 10)
out = torch.empty(n + n // 8 + (1 << 20), dtype=torch.uint8, device="cuda")
for _ in range(2):
    ctx.compress_device(x.data_ptr(), n, out.data_ptr(), out.numel())
torch.cuda.synchronize()
L = bz2mi.lib()
buf = (ctypes.c_ulonglong * 16)()
for k, name in [(0, "huffman"), (1, "bwt"), (2, "mtf"), (3, "fe_chain windows")]:
    r = L.bz2mi_debug_phases(k, buf)
    v = list(buf)
    n_ = max(i for i in range(16) if v[i]) if any(v) else 0
    print(name, "rc", r, "us:", [round((v[i + 1] - v[i]) / 100.0, 1) for i in range(n_) if v[i] and v[i + 1]],
          "total", round((v[n_] - v[0]) / 100.0, 1) if n_ else None)
L.bz2mi_debug_phases(0, buf)
v = list(buf)
print("huffman raw us from slot 0:", [round((x - v[0]) / 100.0, 1) if x else None for x in v])
L.bz2mi_debug_phases(3, buf)
v = list(buf)
print("fe sums (us): table", v[6] / 100.0, "chase", v[7] / 100.0, "bnd", v[8] / 100.0, "slow", v[9] / 100.0, "ends out", v[10], "mid", v[11])
print("fe raw: rounds", v[12], "k", v[13], "slow", v[14], "us to end", round((v[15] - v[0]) / 100.0, 1))
print("timings", ctx.timings())
L.bz2mi_debug_phases(8, buf)
v = list(buf)
if v[8]:
    print("bwt_block_kernel per block (us): text+hist %.1f pair %.1f scatter %.1f children %.1f batches %.1f; blocks %d, batches/block %.1f, pair buckets/block %.2f"
          % tuple([v[k] / 100.0 / v[8] for k in range(5)] + [v[8], v[9] / v[8], v[10] / v[8]]))
if v[8]:
    nb64 = max(1, v[8] // 64)
    print("batch sorts of every 64th block, wave-us per block: sub-buckets %.1f counting %.1f big %.1f whole-segment %.1f"
          % tuple(v[k] / 100.0 / nb64 for k in (11, 12, 13, 14)))
