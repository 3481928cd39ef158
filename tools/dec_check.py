"""Quick device-decoder check: round trips of a few seeded inputs (prints
per-case status; no pytest)."""
import os, sys, traceback, bz2
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bzip2-opencl_amd"))
import bz2mi
from bz2mi import synth
d = bz2mi.Decompressor(10000)
cases = [("empty", b""), ("one", b"x"), ("abc", b"abcabcabd" * 10), ("text", synth.text_bytes(300000).tobytes()),
         ("random", synth.random_bytes(300000).tobytes()), ("runs", synth.runs_bytes(300000).tobytes()),
         ("zeros", bytes(100000))]
for name, data in cases:
    try:
        z = bz2mi.compress(data, 9, 10)
        got = d.decompress(z)
        ok = got == data
        first = next((i for i in range(min(len(got), len(data))) if got[i] != data[i]), None)
        print(name, "ok" if ok else f"MISMATCH len {len(got)} vs {len(data)} first diff {first}", d.timings(), flush=True)
    except Exception as e:
        print(name, "ERROR", repr(e), flush=True)
