"""Issue utilisation of the bz2mi kernels from one rocprofv3 --pmc pass
(tools/r4_measure.sh: SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE, kernel trace only).

Per kernel, summed over its dispatches:
* valu_issue_frac = SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction
  occupies its SIMD-32 for 2 cycles, MI355X_MICROARCH.md) / (1024 SIMDs x the
  kernel's cycles), cycles = GRBM_GUI_ACTIVE / 8 (the counter is summed over
  the 8 XCDs, the guide's effective-clock note), so the quotient is the share
  of SIMD issue slots the kernel's VALU stream used;
* lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (cycles
  lost to bank conflicts over LDS-active cycles);
* eff_clock_GHz = GRBM_GUI_ACTIVE / 8 / wall time of the dispatches.
Writes profiles/<name>.json, read by bench.py for roofline.issue."""
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

src = sys.argv[1]
dst = sys.argv[2]
what = sys.argv[3] if len(sys.argv) > 3 else ""
SIMDS = 256 * 4
acc = collections.defaultdict(lambda: collections.defaultdict(float))
seen = collections.defaultdict(set)
for r in csv.DictReader(open(src)):
    if "bz2mi::" not in r["Kernel_Name"]:
        continue
    k = r["Kernel_Name"].split("(")[0].replace("bz2mi::", "").replace("void ", "")
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    d = r["Dispatch_Id"]
    if d not in seen[k]:
        seen[k].add(d)
        acc[k]["_ns"] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        acc[k]["_n"] += 1
out = {"source": src.split("/")[-1], "what": what, "kernels": {}}
for k, c in sorted(acc.items()):
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    e = {"dispatches": int(c["_n"]), "ms_total": round(c["_ns"] * 1e-6, 3)}
    if cyc > 0:
        e["eff_clock_GHz"] = round(cyc / c["_ns"], 3) if c["_ns"] > 0 else None
        e["valu_issue_frac"] = round(c.get("SQ_INSTS_VALU", 0.0) * 2.0 / (SIMDS * cyc), 4)
        e["salu_per_valu"] = round(c.get("SQ_INSTS_SALU", 0.0) / max(1.0, c.get("SQ_INSTS_VALU", 0.0)), 3)
        e["lds_insts_per_valu"] = round(c.get("SQ_INSTS_LDS", 0.0) / max(1.0, c.get("SQ_INSTS_VALU", 0.0)), 3)
    if c.get("SQ_LDS_IDX_ACTIVE", 0.0) > 0:
        e["lds_bank_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"], 4)
    out["kernels"][k] = e
out["lib_sha16"] = _lib_sha16()
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out["kernels"], indent=1))
