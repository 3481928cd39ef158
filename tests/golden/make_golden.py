#!/usr/bin/env python3
"""Regenerate the committed golden fixtures from O_ref.

O_ref is the reference's own compressor (kernel.cpp device program plus
BlockCompressor.hpp / BitOutputStream.hpp / CRC32.hpp host code) compiled from
/root/reference by oracle/Makefile into oracle/_ref/liboref.so.  This script
only runs where that library exists (the build container); the fixtures it
writes are data -- seeded inputs and the reference's outputs -- so the GPU box
and later rounds can check parity without the reference tree.

Writes, under tests/golden/:
  inputs/<case>.bin                       input bytes
  oref/<case>.s<level>.p<p>.bz2           O_ref compressed stream
  blocks/<case>.s<level>.npz              per-block intermediates of O_ref:
        rle1 (concatenated RLE1 blocks), lens, bwt, orig, mtf, mtflen, alpha
  manifest.json                           sha256 of every file + case metadata
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "bzip2-opencl_amd"))
from bz2mi import synth  # noqa: E402

OREF = os.path.join(REPO, "oracle", "_ref", "liboref.so")
CREF = os.path.join(REPO, "oracle", "_build", "libcpuref.so")


def load():
    o = ctypes.CDLL(OREF)
    o.oref_compress.restype = ctypes.c_longlong
    o.oref_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    o.oref_bwt.restype = ctypes.c_int
    o.oref_bwt.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]
    o.oref_mtf.restype = ctypes.c_int
    o.oref_mtf.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                           ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                           ctypes.POINTER(ctypes.c_int)]
    c = ctypes.CDLL(CREF)
    c.cpuref_split.restype = ctypes.c_longlong
    c.cpuref_split.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_char_p,
                               ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_size_t]
    return o, c


def oref_compress(o, data: bytes, level: int, p: int, unit: int = 10000) -> bytes:
    cap = len(data) * 3 + 100000
    buf = ctypes.create_string_buffer(cap)
    n = o.oref_compress(data, len(data), level, p, unit, buf, cap)
    assert n >= 0, n
    return buf.raw[:n]


def split(c, data: bytes, S: int):
    nb = c.cpuref_split(data, len(data), S, None, 0, None, None, None, 0)
    nb = -nb if nb < 0 else nb
    stride = S + 8
    blocks = ctypes.create_string_buffer(max(1, nb * stride))
    lens = (ctypes.c_uint32 * max(1, nb))()
    c.cpuref_split(data, len(data), S, blocks, stride, None, lens, None, nb)
    return [blocks.raw[b * stride: b * stride + lens[b]] for b in range(nb)]


def period(t: bytes) -> int:
    """Smallest period p < n with t == t[:p] * (n/p), or 0 if aperiodic."""
    n = len(t)
    if n < 2:
        return 0
    for per in range(1, n // 2 + 1):
        if n % per == 0 and t == t[:per] * (n // per):
            return per
    return 0


def cases():
    yield "empty", b""
    yield "one", b"a"
    yield "two_same", b"aa"
    yield "short", b"abcxyz"
    yield "all_bytes", bytes(range(256))
    yield "run255", b"a" * 255
    yield "run256", b"a" * 256
    yield "run259", b"a" * 259
    yield "fb_const", b"\xfb" * 600000          # RLE1 output has constant blocks (H8)
    yield "c1_text10k", synth.text_bytes(10240, synth.SEED_TEXT ^ 1).tobytes()  # config C1
    yield "text64k", synth.text_bytes(65536).tobytes()
    yield "rnd64k", synth.random_bytes(65536).tobytes()
    yield "runs64k", synth.runs_bytes(65536).tobytes()
    yield "acgt64k", synth.small_alphabet_bytes(65536).tobytes()
    # round 4: enwik9-like text (~150 distinct bytes, markup, UTF-8) -- C3
    yield "rtext64k", synth.realtext_bytes(65536).tobytes()
    # a block whose RLE1 length reaches exactly S at -1 (H1)
    yield "h1_exact", find_h1()


def find_h1() -> bytes:
    _, c = load()
    for seed in range(1, 400):
        d = synth.runs_bytes(40000, seed=seed, max_run=8).tobytes()
        if any(len(b) == 10000 for b in split(c, d, 10000)[:-1]):
            return d
    raise RuntimeError("no H1 case found")


def main():
    o, c = load()
    os.makedirs(os.path.join(HERE, "inputs"), exist_ok=True)
    os.makedirs(os.path.join(HERE, "oref"), exist_ok=True)
    os.makedirs(os.path.join(HERE, "blocks"), exist_ok=True)
    manifest = {"generator": "tests/golden/make_golden.py", "oracle": "O_ref (oracle/_ref/liboref.so)",
                "cases": {}, "sha256": {}}

    def put(rel, data: bytes):
        with open(os.path.join(HERE, rel), "wb") as f:
            f.write(data)
        manifest["sha256"][rel] = hashlib.sha256(data).hexdigest()

    for name, data in cases():
        put(f"inputs/{name}.bin", data)
        # constant blocks (period 1) are handled correctly by the reference by
        # accident (H8: its BWT array holds indices, all mapping to symbol 0), so
        # their streams are parity targets but their O_ref BWT bytes are not;
        # blocks with a period >= 2 are wrong in the reference (H2).
        entry = {"n": len(data), "streams": [], "constant_blocks": [], "periodic_blocks": []}
        for level, p in [(1, 1), (1, 10), (9, 1), (9, 10), (9, 3)]:
            rel = f"oref/{name}.s{level}.p{p}.bz2"
            put(rel, oref_compress(o, data, level, p))
            entry["streams"].append({"file": rel, "level": level, "p": p})
        for level in (1, 9):
            blocks = split(c, data, 10000 * level)
            pers = [period(b) for b in blocks]
            entry["constant_blocks"].append({"level": level, "blocks": [i for i, q in enumerate(pers) if q == 1]})
            entry["periodic_blocks"].append({"level": level, "blocks": [i for i, q in enumerate(pers) if q >= 2]})
            if not blocks:
                continue
            lens = np.array([len(b) for b in blocks], dtype=np.int64)
            rle1 = np.frombuffer(b"".join(blocks), dtype=np.uint8)
            bwts, origs, mtfs, mtflen, alphas = [], [], [], [], []
            for b in blocks:
                out = ctypes.create_string_buffer(max(1, len(b)))
                orig = o.oref_bwt(b, len(b), out)
                bw = out.raw[: len(b)]
                present = bytes(1 if v in set(b) else 0 for v in range(256))
                freq = (ctypes.c_int * 258)()
                mtf = (ctypes.c_int * (len(b) + 2))()
                alpha = ctypes.c_int(0)
                m = o.oref_mtf(bw, len(b), present, freq, mtf, ctypes.byref(alpha))
                bwts.append(np.frombuffer(bw, dtype=np.uint8))
                origs.append(orig)
                mtfs.append(np.array(mtf[:m], dtype=np.uint16))
                mtflen.append(m)
                alphas.append(alpha.value)
            rel = f"blocks/{name}.s{level}.npz"
            path = os.path.join(HERE, rel)
            np.savez_compressed(path, rle1=rle1, lens=lens, bwt=np.concatenate(bwts),
                                orig=np.array(origs, dtype=np.int64),
                                mtf=np.concatenate(mtfs), mtflen=np.array(mtflen, dtype=np.int64),
                                alpha=np.array(alphas, dtype=np.int64))
            with open(path, "rb") as f:
                manifest["sha256"][rel] = hashlib.sha256(f.read()).hexdigest()
        manifest["cases"][name] = entry
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", len(manifest["sha256"]), "files")


if __name__ == "__main__":
    main()
