"""The oracle is pinned before it is trusted (CPU only).

* cpu_ref (oracle/cpu_ref.c, the C restatement) reproduces every committed
  O_ref stream byte for byte, at -1 and -9, p in {1, 3, 10};
* its BWT and MTF/RLE2 stages match the per-block O_ref intermediates;
* where O_ref itself can be built (this container), it still reproduces the
  fixtures;
* every fixture stream is valid bzip2 (system bzip2 decodes it to the input).
"""
from __future__ import annotations

import bz2
import os
import random
import shutil
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REPO, golden_file, golden_input, oref_lib


def _cases(manifest):
    for name, e in sorted(manifest["cases"].items()):
        for st in e["streams"]:
            yield name, st["level"], st["p"], st["file"]


def test_manifest_hashes(manifest):
    import hashlib
    for rel, h in manifest["sha256"].items():
        with open(os.path.join(GOLDEN, rel), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == h, rel


def test_cpuref_matches_oref_fixtures(manifest, cpuref):
    for name, level, p, rel in _cases(manifest):
        data = golden_input(name)
        assert cpuref.compress(data, level, p) == golden_file(rel), (name, level, p)


def test_fixture_streams_are_valid_bzip2(manifest):
    for name, level, p, rel in _cases(manifest):
        assert bz2.decompress(golden_file(rel)) == golden_input(name), (name, level, p)


def test_cpuref_stage_intermediates(manifest, cpuref):
    """BWT (+origPtr) and MTF/RLE2 symbols per block against O_ref's."""
    for name, e in sorted(manifest["cases"].items()):
        for level in (1, 9):
            path = os.path.join(GOLDEN, "blocks", f"{name}.s{level}.npz")
            if not os.path.exists(path):
                continue
            z = np.load(path)  # allow_pickle stays False
            const = next(c["blocks"] for c in e["constant_blocks"] if c["level"] == level)
            lens = z["lens"]
            offs = np.concatenate([[0], np.cumsum(lens)])
            moffs = np.concatenate([[0], np.cumsum(z["mtflen"])])
            data = golden_input(name)
            blocks, _ = cpuref.split(data, 10000 * level)
            assert [len(b) for b in blocks] == list(lens)
            for b, blk in enumerate(blocks):
                assert blk == z["rle1"][offs[b]:offs[b + 1]].tobytes()
                bw, orig = cpuref.bwt(blk)
                if b not in const:  # H8: the reference's BWT array holds indices for constant blocks
                    assert bw == z["bwt"][offs[b]:offs[b + 1]].tobytes(), (name, level, b)
                    assert orig == z["orig"][b]
                present = bytes(1 if v in set(blk) else 0 for v in range(256))
                sym, hist, alpha = cpuref.mtf(bw, present)
                assert alpha == z["alpha"][b]
                assert np.array_equal(sym, z["mtf"][moffs[b]:moffs[b + 1]]), (name, level, b)
                assert int(hist.sum()) == len(sym)


@pytest.mark.skipif(oref_lib() is None, reason="O_ref needs /root/reference (build container only)")
def test_oref_still_reproduces_fixtures(manifest):
    import ctypes
    L = oref_lib()
    for name, level, p, rel in _cases(manifest):
        data = golden_input(name)
        cap = len(data) * 3 + 100000
        out = ctypes.create_string_buffer(cap)
        n = L.oref_compress(data, len(data), level, p, 10000, out, cap)
        assert out.raw[:n] == golden_file(rel)


@pytest.mark.skipif(oref_lib() is None, reason="O_ref needs /root/reference (build container only)")
def test_cpuref_matches_oref_random_inputs(cpuref):
    """Seeded property sweep: cpu_ref == O_ref on aperiodic inputs of many shapes."""
    import ctypes
    L = oref_lib()
    rng = random.Random(0x5EED)
    for trial in range(24):
        kind = trial % 4
        n = rng.choice([1, 2, 7, 100, 999, 10000, 30000, 70000])
        if kind == 0:
            data = bytes(rng.getrandbits(8) for _ in range(n))
        elif kind == 1:
            data = bytes(rng.choice(b"abc ") for _ in range(n))
        elif kind == 2:
            out = bytearray()
            while len(out) < n:
                out += bytes([rng.getrandbits(8)]) * rng.randint(1, 300)
            data = bytes(out[:n])
        else:
            data = bytes(rng.choice(b"\x00\x01\xff") for _ in range(n))
        level, p = rng.choice([(1, 1), (1, 10), (2, 3), (9, 10)])
        blocks, _ = cpuref.split(data, 10000 * level)
        if any(_periodic(b) for b in blocks):
            continue  # H2: the reference is wrong on periodic blocks
        cap = len(data) * 3 + 100000
        buf = ctypes.create_string_buffer(cap)
        m = L.oref_compress(data, len(data), level, p, 10000, buf, cap)
        assert cpuref.compress(data, level, p) == buf.raw[:m], (trial, n, level, p)


def _periodic(t: bytes) -> bool:
    n = len(t)
    for q in range(2, n // 2 + 1):
        if n % q == 0 and t == t[:q] * (n // q):
            return True
    return False


def test_cpuref_periodic_blocks_are_valid(cpuref):
    """H2: periodic blocks are outside parity; our tie rule must still decode."""
    for pat, n in [(b"ab", 50000), (b"abc", 30000), (b"the quick brown fox ", 200000), (b"xyzzy", 90000)]:
        data = (pat * (n // len(pat) + 1))[:n]
        for level in (1, 9):
            assert bz2.decompress(cpuref.compress(data, level, 10)) == data


def test_cpuref_900k_mode_is_valid(cpuref):
    rng = np.random.Generator(np.random.PCG64(7))
    data = rng.integers(0, 40, size=2_500_000, dtype=np.uint8).tobytes()
    out = cpuref.compress(data, 9, 10, unit=100000)
    assert out[:4] == b"BZh9"
    assert bz2.decompress(out) == data


@pytest.mark.skipif(shutil.which("bzip2") is None, reason="no system bzip2")
def test_system_bzip2_accepts_cpuref(tmp_path, cpuref):
    data = golden_input("text64k")
    p = tmp_path / "t.bz2"
    p.write_bytes(cpuref.compress(data, 9, 10))
    r = subprocess.run(["bzip2", "-t", str(p)], capture_output=True)
    assert r.returncode == 0, r.stderr


def _asan_cli() -> str:
    exe = os.path.join(REPO, "oracle", "_build", "cpuref_cli_asan")
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "asan"], check=True, stdout=subprocess.DEVNULL,
                   stderr=subprocess.DEVNULL)
    return exe


def test_cpuref_under_asan_ubsan(manifest, tmp_path):
    """The checker itself under AddressSanitizer + UndefinedBehaviorSanitizer
    (oracle/Makefile `asan`): every golden fixture at every
    committed setting, single-threaded and on the pthread pool, and two of the
    pins' multi-block inputs (seed slots reused, runs across blocks), must
    reproduce the O_ref bytes with no sanitizer report."""
    import hashlib
    import sys
    sys.path.insert(0, GOLDEN)
    import make_pins
    import json
    exe = _asan_cli()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    src, dst = tmp_path / "in.bin", tmp_path / "out.bz2"

    def run(data: bytes, level: int, p: int, unit: int = 10000, threads: int = 1) -> bytes:
        src.write_bytes(data)
        r = subprocess.run([exe, str(src), str(dst), "-s", str(level), "-p", str(p), "-u", str(unit),
                            "-j", str(threads)], capture_output=True, text=True, env=env, timeout=600)
        assert r.returncode == 0 and "runtime error" not in r.stderr and "ERROR" not in r.stderr, r.stderr[-2000:]
        return dst.read_bytes()

    for i, (name, level, p, file) in enumerate(_cases(manifest)):
        assert run(golden_input(name), level, p, threads=1 + (i & 1)) == golden_file(file), file
    with open(os.path.join(GOLDEN, "pins.json")) as f:
        pins = json.load(f)
    want = {(p["input"], p["level"], p["p"], p["unit"]): (p["bytes"], p["sha256"]) for p in pins["pins"]}
    for key in (("mix2m75", 9, 10, 10000), ("run2m75", 9, 3, 10000)):
        assert key in want, key
        got = run(make_pins.make_input(key[0]), key[1], key[2], key[3], threads=2)
        assert (len(got), hashlib.sha256(got).hexdigest()) == want[key], key
