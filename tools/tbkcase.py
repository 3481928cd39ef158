"""Debug: one golden case (name level p) through the device path, timed."""
import os, sys, time
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(R, "bzip2-opencl_amd"))
sys.path.insert(0, os.path.join(R, "tests"))
import bz2mi
from conftest import golden_input, golden_file
name, level, p = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
data = golden_input(name)
t0 = time.time()
got = bz2mi.compress(data, level, p)
print(os.path.basename(os.environ.get("BZ2MI_LIBRARY", "main")), name, level, p,
      got == golden_file(f"oref/{name}.s{level}.p{p}.bz2"), round(time.time() - t0, 3), flush=True)
