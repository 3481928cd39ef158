"""Collect the reference-on-MI355X streams of tools/ref_opencl3.sh
(gpurun_out/refcl3/) into tests/golden/refgpu/ and refgpu.json (input
descriptors as tests/test_refgpu.py reads them)."""
import hashlib
import json
import os
import re
import shutil
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(R, "gpurun_out", "refcl3")
INPUTS = {
    "rtext64k": ("golden:rtext64k", 65536),
    "rtx2m75": ("pins:rtx2m75", 2883584),
    "rep2m75": ("pins:rep2m75", 2883584),
    "rep64k": ("synth:repeats:65536", 65536),
    "rep1m": ("synth:repeats:1048576", 1 << 20),
    "rtx1m": ("synth:realtext:1048576:0x5EED3001", 1 << 20),
}
js = os.path.join(R, "tests", "golden", "refgpu.json")
d = json.load(open(js))
have = {e["file"] for e in d["streams"]}
times = {}
for line in open(os.path.join(src, "times.txt")):
    m = re.match(r"(\S+)\.bin -s (\d) -p (\d+) rc=0 ms=(\d+)", line)
    if m:
        times[(m.group(1), int(m.group(2)), int(m.group(3)))] = int(m.group(4))
for (name, level, p), ms in sorted(times.items()):
    f = f"{name}.bin.s{level}.p{p}.bz2"
    z = open(os.path.join(src, "w", f), "rb").read()
    rel = f"refgpu/{name}.s{level}.p{p}.bz2"
    shutil.copy(os.path.join(src, "w", f), os.path.join(R, "tests", "golden", rel))
    e = {"bytes": len(z), "file": rel, "input": INPUTS[name][0], "input_bytes": INPUTS[name][1], "level": level,
         "p": p, "process_ms": ms, "sha256": hashlib.sha256(z).hexdigest(), "round": 5}
    if rel in have:
        d["streams"] = [x for x in d["streams"] if x["file"] != rel]
    d["streams"].append(e)
    print(rel, len(z), ms)
d["streams"].sort(key=lambda e: e["file"])
d["generator_r5"] = ("tools/ref_opencl3.sh (the same unmodified reference build, round 5: wide-alphabet text and "
                     "deep repeats)")
json.dump(d, open(js, "w"), indent=1, sort_keys=True)
