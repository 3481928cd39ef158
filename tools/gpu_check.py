"""Quick GPU parity probe: golden streams + per-block payloads vs cpu_ref."""
import ctypes, json, os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "bzip2-opencl_amd"))
import bz2mi
from bz2mi import synth

G = os.path.join(REPO, "tests", "golden")
man = json.load(open(os.path.join(G, "manifest.json")))
bad = 0
for name, e in sorted(man["cases"].items()):
    data = open(os.path.join(G, "inputs", name + ".bin"), "rb").read()
    for st in e["streams"]:
        ref = open(os.path.join(G, st["file"]), "rb").read()
        t = time.time()
        got = bz2mi.compress(data, st["level"], st["p"])
        ok = got == ref
        bad += not ok
        print(f"{name:12s} s{st['level']} p{st['p']:2d} ref={len(ref):7d} gpu={len(got):7d} {'OK' if ok else 'DIFF'} {time.time()-t:.2f}s", flush=True)
        if not ok:
            n = min(len(ref), len(got)); d = next((i for i in range(n) if ref[i] != got[i]), n)
            print("   first diff byte", d)
cref = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "libcpuref.so"))
cref.cpuref_compress.restype = ctypes.c_longlong
cref.cpuref_bound.restype = ctypes.c_size_t
cases = [(synth.text_bytes, 4 << 20), (synth.random_bytes, 4 << 20), (synth.runs_bytes, 4 << 20),
         (synth.small_alphabet_bytes, 1 << 20),
         (lambda n: np.frombuffer((b"ab" * n)[:n], dtype=np.uint8), 300000),
         (lambda n: np.frombuffer((b"abcab" * n)[:n], dtype=np.uint8), 200000),
         (lambda n: np.frombuffer((b"the quick brown fox " * n)[:n], dtype=np.uint8), 250000)]
for gen, n in cases:
    d = gen(n).tobytes()
    cap = cref.cpuref_bound(ctypes.c_size_t(len(d)), 9, 10000)
    out = ctypes.create_string_buffer(cap)
    r = cref.cpuref_compress(d, ctypes.c_size_t(len(d)), 9, 10, 10000, out, ctypes.c_size_t(cap), 8)
    ref = out.raw[:r]
    t = time.time()
    ctx = bz2mi.Context(9, 10)
    got = ctx.compress(d)
    dt = time.time() - t
    print(getattr(gen, "__name__", "lambda"), len(d), len(ref), len(got), "OK" if got == ref else "DIFF", f"{dt:.2f}s", ctx.timings(), flush=True)
    bad += got != ref
print("BAD", bad)
