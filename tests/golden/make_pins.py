#!/usr/bin/env python3
"""Hash pins of the reference compressor (O_ref) at the headline configuration.

The committed fixtures (make_golden.py) are small: at -9 every one is a single
block, so the per-slot seed carry-over of the reference (its frequency array is
never cleared, OutputStream.hpp:93 / kernel.cpp:3155; slot = block mod p) never
wraps there.  These pins cover it: seeded multi-MiB inputs, regenerated
bit-for-bit from bz2mi.synth at test time, compressed by O_ref
(oracle/_ref/liboref.so, the reference's own kernel.cpp + BlockCompressor /
BitOutputStream / CRC32 compiled from /root/reference) at

  * -9 (S = 90,000), p = 10, 3 and 1 on 2.75 MiB of random, text, mixed and
    run-heavy bytes (32 blocks: every slot of p = 10 is reused three times);
  * -1 (S = 10,000), p = 10 on the same inputs (~290 blocks);
  * O_ref900 (the 900 KB mode, Config.hpp:30 BLOCKSIZE_DEFAULT = 100000):
    -9 at p = 10 and 3 on 12 MiB of random, text and mixed bytes (14 blocks);
  * round 4: the enwik9-like C3 text (synth.realtext_bytes: ~150 distinct
    bytes per 90 KB block) and its long-repeat variant (synth.repeats_bytes)
    at -9 p = 10/3/1 and -1, and the realtext in the 900 KB mode.

Only the SHA-256 and length of each output are stored (tests/golden/pins.json),
with the SHA-256 of the input so generator drift is caught.  Run in the build
container (where O_ref exists) after `make -C oracle ref`.
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "bzip2-opencl_amd"))
from bz2mi import synth  # noqa: E402

OREF = os.path.join(REPO, "oracle", "_ref", "liboref.so")

# name -> (generator, n); the same code regenerates the inputs in the tests
INPUTS = {
    "rnd2m75": ("random", 2_883_584),
    "txt2m75": ("text", 2_883_584),
    "mix2m75": ("mixed", 2_883_584),
    "run2m75": ("runs", 2_883_584),
    "rnd12m": ("random", 12 << 20),
    "txt12m": ("text", 12 << 20),
    "mix12m": ("mixed", 12 << 20),
    "rtx2m75": ("realtext", 2_883_584),
    "rep2m75": ("repeats", 2_883_584),
    "rtx12m": ("realtext", 12 << 20),
}

PINS = [(name, level, p, 10000) for name in ("rnd2m75", "txt2m75", "mix2m75", "run2m75")
        for level, p in ((9, 10), (9, 3), (9, 1), (1, 10))]
PINS += [(name, 9, p, 100000) for name in ("rnd12m", "txt12m", "mix12m") for p in (10, 3)]
# round 4: C3 enwik9-like text (synth.realtext_bytes, ~150 distinct bytes per
# block) and its long-repeat stress variant (synth.repeats_bytes)
PINS += [(name, level, p, 10000) for name in ("rtx2m75", "rep2m75") for level, p in ((9, 10), (9, 3), (9, 1), (1, 10))]
PINS += [("rtx12m", 9, p, 100000) for p in (10, 3)]


def make_input(name: str) -> bytes:
    kind, n = INPUTS[name]
    seed = 0x5EED1000 + sum(map(ord, name))
    if kind == "random":
        return synth.random_bytes(n, seed).tobytes()
    if kind == "text":
        return synth.text_bytes(n, seed).tobytes()
    if kind == "realtext":
        return synth.realtext_bytes(n, seed).tobytes()
    if kind == "repeats":
        return synth.repeats_bytes(n, seed).tobytes()
    if kind == "runs":  # runs of 1..12: RLE1 pieces of every length, ~19 blocks at -9
        return synth.runs_bytes(n, seed, max_run=12).tobytes()
    return synth.mixed_bytes(n, seed, segment=512 << 10).tobytes()


def main():
    o = ctypes.CDLL(OREF)
    o.oref_compress.restype = ctypes.c_longlong
    o.oref_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    inputs = {name: make_input(name) for name in INPUTS}
    out = {"generator": "tests/golden/make_pins.py", "oracle": "O_ref (oracle/_ref/liboref.so)",
           "inputs": {k: {"kind": v[0], "n": v[1], "sha256": hashlib.sha256(inputs[k]).hexdigest()}
                      for k, v in INPUTS.items()},
           "pins": []}
    for name, level, p, unit in PINS:
        data = inputs[name]
        cap = len(data) * 3 + 100000
        buf = ctypes.create_string_buffer(cap)
        t0 = time.time()
        n = o.oref_compress(data, len(data), level, p, unit, buf, cap)
        assert n >= 0, n
        z = buf.raw[:n]
        out["pins"].append({"input": name, "level": level, "p": p, "unit": unit, "bytes": n,
                            "sha256": hashlib.sha256(z).hexdigest()})
        print(f"{name} -{level} p={p} unit={unit}: {n} bytes ({time.time() - t0:.1f} s)")
    with open(os.path.join(HERE, "pins.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
