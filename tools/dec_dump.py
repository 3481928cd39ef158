"""Debug: decode one small stream with BZ2MI_DDUMP and compare the first
block's BWT bytes / origPtr with the C restatement's (cpu_ref)."""
import os, sys, struct
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bzip2-opencl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import bz2mi
from conftest import CpuRef
cr = CpuRef()
data = (b"abcabcabd" * 10) if len(sys.argv) < 2 else open(sys.argv[1], "rb").read()
z = bz2mi.compress(data, 9, 10)
path = "/tmp/ddump.bin"
os.environ["BZ2MI_DDUMP"] = path
d = bz2mi.Decompressor(10000)
try:
    print("decoded ok:", d.decompress(z) == data, flush=True)
except Exception as e:
    print("decode error:", e, flush=True)
raw = open(path, "rb").read()
end_bit, status, orig, ln, crc, nsym, alpha = struct.unpack("<QIIIIII", raw[:32])
got = raw[32:]
blocks, _ = cr.split(data, 90000)
bw, o = cr.bwt(blocks[0])
print("status", status, "orig", orig, "want", o, "len", ln, "want", len(bw), "end_bit", end_bit, flush=True)
bw = bytes(bw)
print("bwt equal:", got == bw[: len(got)], "first diff", next((i for i in range(min(len(got), len(bw))) if got[i] != bw[i]), None))
print("got ", got[:40])
print("want", bw[:40])
os.environ["BZ2MI_DNOCRC"] = "1"
out = d.decompress(z)
print("nocrc output equal:", out == data, len(out), len(data))
print("out ", out[:60])
print("want", data[:60])
