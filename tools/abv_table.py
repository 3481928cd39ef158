"""Table of tools/ab_variants.sh results: value and stage times per variant."""
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/abv"
for f in sorted(glob.glob(os.path.join(root, "*.json"))):
    try:
        d = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable", e)
        continue
    st = d.get("roofline", {}).get("stage_ms", {})
    print("%-24s %9.1f  %s" % (os.path.basename(f)[:-5], d["value"], " ".join("%s=%.2f" % kv for kv in st.items())))
