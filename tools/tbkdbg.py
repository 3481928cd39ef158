"""Debug: every golden input through the device path (BZ2MI_BWT_STATS=1 prints
how the BWT handled the blocks), timed, checked against the O_ref fixtures."""
import json, os, sys, time
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(R, "bzip2-opencl_amd"))
sys.path.insert(0, os.path.join(R, "tests"))
import bz2mi
from conftest import golden_input, golden_file
m = json.load(open(os.path.join(R, "tests", "golden", "manifest.json")))
for name, e in sorted(m["cases"].items()):
    data = golden_input(name)
    for st in e["streams"]:
        t0 = time.time()
        got = bz2mi.compress(data, st["level"], st["p"])
        print(name, st["level"], st["p"], got == golden_file(st["file"]), round(time.time() - t0, 3), flush=True)
