import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bzip2-opencl_amd"))
import bz2mi
for d in [b"a", b"ab", b"aa", b"abc"]:
    print(d, flush=True)
    print(bz2mi.compress(d, 1, 1).hex(), flush=True)
