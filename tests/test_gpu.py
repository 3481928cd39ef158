"""Parity of the HIP path (through the C ABI) on an MI355X.

Every comparison is byte-for-byte: against the committed O_ref fixtures, and
against the C restatement cpu_ref (itself pinned to O_ref by test_oracle.py) on
seeded inputs of every data shape the reference's hazards touch.  At the full
BASELINE size (1 GiB) parity is checked through a size-independent property:
the stream decodes back to the input.
"""
from __future__ import annotations

import bz2
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG, REPO, golden_file, golden_input

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bz():
    import bz2mi
    if bz2mi.lib().bz2mi_device_count() <= 0:
        pytest.fail("no HIP device: the gpu tests need an MI355X")
    return bz2mi


def test_cross_lane_primitives(bz):
    """DPP / permlane moves and DPP wave scans agree with ds_bpermute shuffles
    and serial sums (the sorts and scans of every kernel build on them)."""
    bad = (ctypes.c_uint32 * 16)()
    L = bz.lib()
    assert L.bz2mi_debug_selftest(bad, 16) == 10
    names = ["xor1", "xor2", "xor4", "xor8", "xor16", "xor32", "lane_prev", "incl_sum", "incl_max", "wave_sum"]
    assert {n: bad[i] for i, n in enumerate(names) if bad[i]} == {}, " ".join(str(x) for x in bad)


def test_golden_streams(bz, manifest):
    for name, e in sorted(manifest["cases"].items()):
        data = golden_input(name)
        for st in e["streams"]:
            assert bz.compress(data, st["level"], st["p"]) == golden_file(st["file"]), (name, st)


def _repeats(n: int) -> np.ndarray:
    from bz2mi import synth
    return synth.repeats_bytes(n)


def _random_repeats(n: int, seed: int = 0x5EED0909) -> np.ndarray:
    """Random bytes with copies of earlier stretches (64 B .. 6 KB): blocks of
    random-like first-byte buckets whose rotations tie far past the tie
    kernels' depth, so the block path's groups reach prefix doubling (the
    second pass of bwt_block_kernel writes their final SA entries)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    x = rng.integers(0, 256, size=n, dtype=np.uint8)
    p = 20_000
    while p < n - 7000:
        ln = int(rng.choice([64, 300, 1500, 6000]))
        src = int(rng.integers(max(0, p - 60_000), p - ln))
        x[p:p + ln] = x[src:src + ln]
        p += ln + int(rng.integers(2_000, 40_000))
    return x


def _inputs():
    from bz2mi import synth
    yield "random_repeats", _random_repeats(3 << 20)
    yield "text", synth.text_bytes(6 << 20)
    yield "realtext", synth.realtext_bytes(6 << 20)
    yield "realtext_repeats", _repeats(4 << 20)
    yield "random", synth.random_bytes(6 << 20)
    yield "runs", synth.runs_bytes(6 << 20)
    yield "acgt", synth.small_alphabet_bytes(3 << 20)
    yield "mixed", synth.mixed_bytes(8 << 20, segment=1 << 20)
    yield "runs_long", synth.runs_bytes(4 << 20, max_run=5000)
    yield "zeros", np.zeros(3 << 20, dtype=np.uint8)
    yield "periodic_ab", np.frombuffer(b"ab" * (1 << 19), dtype=np.uint8)
    yield "periodic_sentence", np.frombuffer(b"the quick brown fox jumps " * 40000, dtype=np.uint8)


@pytest.mark.parametrize("level,p", [(9, 10), (1, 1), (5, 3)])
def test_seeded_inputs_match_cpuref(bz, cpuref, level, p):
    for name, arr in _inputs():
        data = arr.tobytes()
        want = cpuref.compress(data, level, p, threads=16)
        got = bz.compress(data, level, p)
        assert got == want, (name, level, p, len(got), len(want))


def test_900k_mode_matches_cpuref(bz, cpuref):
    from bz2mi import synth
    for data in (synth.text_bytes(5 << 20).tobytes(), synth.random_bytes(3 << 20).tobytes(),
                 synth.realtext_bytes(6 << 20).tobytes(), _repeats(4 << 20).tobytes()):
        want = cpuref.compress(data, 9, 10, unit=100000, threads=16)
        got = bz.compress(data, 9, 10, unit=100000)
        assert got == want
        assert bz2.decompress(got) == data


@pytest.mark.parametrize("level", [9, 1])
def test_900k_mode_periodic_and_small_alphabets_match_cpuref(bz, cpuref, level):
    """Blocks beyond the LDS text (unit 100000) whose tie groups reach the
    grid-wide doubling's large-group path (periodic blocks: groups of n /
    period rotations, doubling to h >= n) and its repeat pairs."""
    from bz2mi import synth
    rng = np.random.default_rng(0x5EED0905)
    pattern = rng.integers(0, 256, 3000, dtype=np.uint8).tobytes()
    cases = {
        "periodic_ab": b"ab" * (1 << 19),
        "periodic_sentence": b"the quick brown fox jumps " * 40000,
        "periodic_3000": pattern * 700,
        "acgt": synth.small_alphabet_bytes(2 << 20).tobytes(),
        "zeros": bytes(3 << 20),
        "mixed": synth.mixed_bytes(4 << 20, segment=512 << 10).tobytes(),
    }
    for name, data in cases.items():
        want = cpuref.compress(data, level, 10, unit=100000, threads=16)
        got = bz.compress(data, level, 10, unit=100000)
        assert got == want, (name, level)
        assert bz2.decompress(got) == data, name


def test_small_batches_carry_state(bz, cpuref):
    """Back-end batches of 7 blocks: seed carry-over and bit carry across calls."""
    from bz2mi import synth
    data = synth.mixed_bytes(3 << 20, segment=256 << 10).tobytes()
    os.environ["BZ2MI_BATCH_BLOCKS"] = "7"
    try:
        got = bz.compress(data, 9, 10)
    finally:
        del os.environ["BZ2MI_BATCH_BLOCKS"]
    assert got == cpuref.compress(data, 9, 10, threads=16)


def test_block_api_matches_cpuref_payloads(bz, cpuref):
    """bz2mi_compress_blocks (the kernel_close analogue) vs cpuref_block_payload."""
    from bz2mi import synth
    data = synth.text_bytes(1 << 20).tobytes()
    blocks, _ = cpuref.split(data, 90000)
    ctx = bz.Context(9, 10)
    got = ctx.compress_blocks(blocks)
    seeds = np.zeros((len(blocks), 258), dtype=np.uint32)
    acc = np.zeros((10, 258), dtype=np.uint32)
    for b, blk in enumerate(blocks):
        bw, orig = cpuref.bwt(blk)
        present = bytes(1 if v in set(blk) else 0 for v in range(256))
        sym, hist, alpha = cpuref.mtf(bw, present)
        acc[b % 10] += hist
        cap = 4 << 20
        out = ctypes.create_string_buffer(cap)
        nbits = cpuref.L.cpuref_block_payload(orig, present, sym.ctypes.data, len(sym), alpha,
                                              acc[b % 10].ctypes.data, out, cap * 8, None, None)
        assert got[b][1] == nbits
        assert got[b][0] == out.raw[: (nbits + 7) // 8], b


def test_device_api_and_context_reuse(bz):
    import torch
    from bz2mi import synth
    data = synth.text_bytes(3 << 20)
    ctx = bz.Context(9, 10)
    x = torch.from_numpy(data).cuda()
    cap = bz.compress_bound(len(data))
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    n1 = ctx.compress_device(x.data_ptr(), len(data), out.data_ptr(), cap)
    s1 = out[:n1].cpu().numpy().tobytes()
    n2 = ctx.compress_device(x.data_ptr(), len(data), out.data_ptr(), cap)
    s2 = out[:n2].cpu().numpy().tobytes()
    assert s1 == s2 == bz.compress(data.tobytes(), 9, 10)


def test_input_written_on_null_stream_without_sync(bz):
    """compress_device with stream 0 orders itself after the input's writers
    on the null stream (where torch works by default): the input is still being
    rewritten by queued kernels when the call is made -- no synchronize and no
    allocation in between (the non-blocking streams must wait)."""
    import torch
    n = 64 << 20
    rng = np.random.default_rng(0x5EED0042)
    base = rng.integers(0, 256, n, dtype=np.uint8)
    ctx = bz.Context(9, 10)
    cap = bz.compress_bound(n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    x = torch.from_numpy(base).cuda()
    torch.cuda.synchronize()
    for _ in range(21):  # an odd number of passes: x = base ^ 0x5A at the end
        x.bitwise_xor_(0x5A)
    m = ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)
    got = out[:m].cpu().numpy().tobytes()
    assert got == bz.compress((base ^ np.uint8(0x5A)).tobytes(), 9, 10)


def test_full_size_random_round_trip(bz, cpuref):
    """BASELINE config C2 at full size: the 1 GiB stream at -9, p = 10 is the C
    restatement's (cpu_ref on the host's cores, pinned to O_ref) byte for
    byte, and decodes back with libbz2."""
    import torch
    n = 1 << 30
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0001)
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    cap = bz.compress_bound(n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    ctx = bz.Context(9, 10)
    m = ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)
    stream = out[:m].cpu().numpy().tobytes()
    del out
    assert stream[:4] == b"BZh9"
    host = x.cpu().numpy().tobytes()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    assert stream == cpuref.compress(host, 9, 10, threads=threads)
    assert bz2.decompress(stream) == host


OS_HARNESS = r"""
#include <fstream>
#include <iostream>
#include <sstream>
#include "OutputStream.hpp"
int main(int argc, char** argv) {
    std::ifstream f(argv[1], std::ios::binary);
    std::stringstream ss; ss << f.rdbuf();
    std::string in = ss.str();
    std::ofstream o(argv[2], std::ios::binary);
    OutputStream s(o, std::atoi(argv[3]), std::atoi(argv[4]));
    if (argc > 5) { std::vector<char> v(in.begin(), in.end()); s.write(v, 0, (int)v.size()); }
    else for (char c : in) s.write(c);
    s.close();
    try { s.write(1); return 3; } catch (const std::runtime_error&) {}
    return 0;
}
"""


def test_outputstream_mirror_matches_cpuref(bz, cpuref, tmp_path):
    src = tmp_path / "os.cpp"
    src.write_text(OS_HARNESS)
    exe = tmp_path / "os"
    lib = os.path.join(PKG, "bz2mi")
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(PKG, "include"), "-I",
                    os.path.join(REPO, "include"), str(src), "-o", str(exe), "-L", lib, "-lbz2mi",
                    "-Wl,-rpath," + lib], check=True)
    from bz2mi import synth
    data = synth.mixed_bytes(2 << 20, segment=300_000).tobytes()
    inp = tmp_path / "in.bin"
    inp.write_bytes(data)
    for level, p, vec in [(9, 10, False), (1, 3, True)]:
        outp = tmp_path / "out.bz2"
        args = [str(exe), str(inp), str(outp), str(level), str(p)] + (["v"] if vec else [])
        r = subprocess.run(args, capture_output=True)
        assert r.returncode == 0, r.stderr
        assert outp.read_bytes() == cpuref.compress(data, level, p, threads=16)


def _no_runs(n: int, seed: int) -> bytes:
    """Random bytes with no two neighbours equal: no RLE1 runs, so the raw
    bytes are the RLE1 bytes and block boundaries are easy to place."""
    rng = np.random.default_rng(seed)
    d = rng.integers(1, 256, n, dtype=np.int64)
    return (np.cumsum(d) % 256).astype(np.uint8).tobytes()


@pytest.mark.parametrize("level", [9, 1])
def test_900k_mode_tiny_blocks_match_cpuref(bz, cpuref, level):
    """Blocks of 0/1 bytes in the 900 KB mode (the big-bucket count
    of a 1-byte block was left unwritten): a 1-byte stream, a 2-byte stream, and
    a stream whose last block is exactly 1 byte, in one batch with many full
    blocks and on their own -- equal to cpu_ref and decoding back."""
    S = level * 100000
    base = _no_runs(3 * S, 0x5EED0906)
    blocks, _ = cpuref.split(base, S)
    n0 = len(blocks[0])
    tail1 = base[: n0 + 1]
    assert [len(b) for b in cpuref.split(tail1, S)[0]] == [n0, 1]
    tail1_many = base[: 2 * n0 + 1]
    assert [len(b) for b in cpuref.split(tail1_many, S)[0]] == [n0, n0, 1]
    for name, data in {"one": b"x", "two": b"xy", "tail1": tail1, "tail1_many": tail1_many}.items():
        for p in (10, 1):
            got = bz.compress(data, level, p, unit=100000)
            assert got == cpuref.compress(data, level, p, unit=100000, threads=16), (name, p)
            assert bz2.decompress(got) == data, name
    # a context reused after a wide block: a 1-byte block must not see its predecessor's lists
    ctx = bz.Context(level, 10, 100000)
    for data in (base, b"z", tail1, b"q"):
        assert ctx.compress(data) == cpuref.compress(data, level, 10, unit=100000, threads=16)


@pytest.mark.timeout(600)
def test_900k_mode_random_1gib_matches_cpuref(bz, cpuref):
    """The bench's mode_900k workload at its own size: 1 GiB of random bytes
    (the C2 seed) at -9 in the 900 KB mode, one batch of 1,194 blocks through
    the big-bucket kernel and the grid doubling -- the C restatement's stream
    byte for byte, decoding back on the device."""
    import torch
    n = 1 << 30
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED0001)
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    cap = bz.compress_bound(n, 9, 100000)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    ctx = bz.Context(9, 10, 100000)
    m = ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)
    stream = out[:m].cpu().numpy().tobytes()
    host = x.cpu().numpy().tobytes()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    assert stream == cpuref.compress(host, 9, 10, unit=100000, threads=threads)
    y = torch.empty(n, dtype=torch.uint8, device="cuda")
    d = bz.Decompressor(100000)
    assert d.decompress_device(out.data_ptr(), m, y.data_ptr(), n) == n
    assert torch.equal(x, y)


def test_900k_mode_under_memory_pressure(bz, cpuref):
    """Most of HBM held by another allocation (all but 16 GiB): the 900 KB
    mode sizes its batches from the free memory (several batches instead of
    one); and with every device allocation above 1 GiB made to fail
    (BZ2MI_DEBUG_MAX_ALLOC), the batches are halved until they fit.  The
    stream stays the C restatement's."""
    import torch
    from bz2mi import synth
    data = synth.random_bytes(256 << 20).tobytes()
    want = cpuref.compress(data, 9, 10, unit=100000, threads=16)
    free, _total = torch.cuda.mem_get_info()
    hold = torch.empty(max(0, free - (16 << 30)), dtype=torch.uint8, device="cuda")
    try:
        assert bz.compress(data, 9, 10, unit=100000) == want
        text = synth.realtext_bytes(24 << 20).tobytes()
        assert bz.compress(text, 9, 10, unit=100000) == cpuref.compress(text, 9, 10, unit=100000, threads=16)
    finally:
        del hold
        torch.cuda.empty_cache()
    os.environ["BZ2MI_DEBUG_MAX_ALLOC"] = str(1 << 30)
    try:
        got = subprocess.run([sys.executable, "-c", "import sys, bz2mi; d = sys.stdin.buffer.read(); "
                              "sys.stdout.buffer.write(bz2mi.compress(d, 9, 10, unit=100000))"],
                             input=data, capture_output=True, cwd=os.path.join(PKG), check=True).stdout
    finally:
        del os.environ["BZ2MI_DEBUG_MAX_ALLOC"]
    assert got == want
