"""Front-end debugging aid: compress golden inputs on the GPU and report where
the stream departs from the committed O_ref fixture (block CRC field vs the
rest), and whether Python's bz2 decodes it back."""
import bz2, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bzip2-opencl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import bz2mi
from conftest import golden_input, golden_file
import json
man = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests/golden/manifest.json")))
for name in sorted(man["cases"]):
    data = golden_input(name)
    for st in man["cases"][name]["streams"]:
        got = bz2mi.compress(data, st["level"], st["p"])
        want = golden_file(st["file"])
        if got == want:
            continue
        first = next((i for i in range(min(len(got), len(want))) if got[i] != want[i]), min(len(got), len(want)))
        try:
            ok = bz2.decompress(got) == data
            dec = "decodes OK" if ok else "decodes to different data"
        except Exception as e:
            dec = f"decode error {e}"
        print(name, st, "len", len(got), len(want), "first diff byte", first, "crc field got", got[10:14].hex(), "want", want[10:14].hex(), dec)
        continue
