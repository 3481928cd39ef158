"""Debug: how the blocks of the random-with-repeats test input go through the
BWT (BZ2MI_BWT_STATS=1 prints the general / text / handed-back split and the
blocks that reach prefix doubling), and parity with the C restatement."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "bzip2-opencl_amd")]
os.environ["BZ2MI_BWT_STATS"] = "1"
import bz2mi
from conftest import CpuRef
from test_gpu import _random_repeats
x = _random_repeats(3 << 20).tobytes()
for level in (9, 1):
    got = bz2mi.compress(x, level, 10)
    print("level", level, "equal", got == CpuRef().compress(x, level, 10, threads=16), flush=True)
