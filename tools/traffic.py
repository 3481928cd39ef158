"""Per-launch HBM-side traffic of the bz2mi kernels from tools/measure.sh's
two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; kB per dispatch).

The bench command of those passes runs 2 compressions (1 warmup + 1 step);
every kernel's counters are averaged over its dispatches per compression.
FETCH_SIZE is doubled as /opt/skills/guides/MI355X_MICROARCH.md prescribes for
gfx950 (it reports half the bytes of wide coalesced reads); WRITE_SIZE is
taken as is.  Both count Infinity-Cache traffic too (the guide).  Writes
profiles/<name>.json, read by bench.py for the `traffic` field."""
import collections
import csv
import json
import os
import sys


def _lib_sha16():
    """the library the measured command loaded (bench.py refuses a profile of another build)"""
    import hashlib
    root = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    path = os.environ.get("BZ2MI_LIBRARY") or os.path.join(root, "bzip2-opencl_amd", "bz2mi", "libbz2mi.so")
    return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/round"
dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/r01_traffic.json"
steps = 2
suffix = sys.argv[3] if len(sys.argv) > 3 else ""  # e.g. "_random" for tools/measure.sh
workload = sys.argv[4] if len(sys.argv) > 4 else "C2"
per = collections.defaultdict(lambda: {"fetch_bytes": 0.0, "write_bytes": 0.0, "dispatches": 0})
for counter, sub, scale in (("FETCH_SIZE", "pmc_fetch", 2.0), ("WRITE_SIZE", "pmc_write", 1.0)):
    for r in csv.DictReader(open(f"{src}/{sub}{suffix}/run_counter_collection.csv")):
        if "bz2mi::" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("bz2mi::", "").replace("void ", "")
        key = "fetch_bytes" if counter == "FETCH_SIZE" else "write_bytes"
        per[k][key] += float(r["Counter_Value"]) * 1024.0 * scale / steps
        if counter == "FETCH_SIZE":
            per[k]["dispatches"] += 1
stages = {"front": ["fe_"], "bwt": ["bwt_", "dbl_"], "mtf": ["mtf_kernel"], "huffman": ["huffman_kernel"],
          "assemble": ["assemble", "offsets_dev", "advance"]}
out = {"command": "python3 bench.py --no-cpu --no-verify --steps 1 --warmup 1 " + (sys.argv[5] if len(sys.argv) > 5 else "") + " (1 GiB, -9, p=10)",
       "workload": workload, "note": "bytes per compression of the 1 GiB input; FETCH_SIZE x2 (gfx950 correction)",
       "kernels": {k: {a: round(b) for a, b in v.items()} for k, v in sorted(per.items())},
       "stages": {}}
for st, pre in stages.items():
    f = sum(v["fetch_bytes"] for k, v in per.items() if any(k.startswith(p) for p in pre))
    w = sum(v["write_bytes"] for k, v in per.items() if any(k.startswith(p) for p in pre))
    out["stages"][st] = {"fetch_bytes": round(f), "write_bytes": round(w), "traffic_bytes": round(f + w)}
out["lib_sha16"] = _lib_sha16()
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out["stages"], indent=1))
