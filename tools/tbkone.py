"""Debug: one golden input through the device path with BZ2MI_BWT_STATS."""
import os, sys, time
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(R, "bzip2-opencl_amd"))
sys.path.insert(0, os.path.join(R, "tests"))
import bz2mi
from conftest import golden_input, golden_file
name = sys.argv[1] if len(sys.argv) > 1 else "text64k"
data = golden_input(name)
t0 = time.time()
got = bz2mi.compress(data, 9, 10)
print(name, got == golden_file(f"oref/{name}.s9.p10.bz2"), round(time.time() - t0, 3), flush=True)
