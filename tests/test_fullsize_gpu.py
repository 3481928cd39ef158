"""Full-size parity of the BASELINE configurations that are not random bytes
(SURVEY.md section 8(d)): C3 (the enwik9 stand-ins: 1 GiB of enwik9-like text,
synth.realtext_bytes, and of seeded word-Markov text, synth.text_bytes)
against the C restatement on the host's cores, and C4
(8 GiB mixed-entropy stream, synth.mixed_bytes) through the unit protocol of
bz2mi.shard -- the path the 8-GPU configuration shards -- against one
compress_device call and back through the device decoder.

Reference: kernel.cpp:3124-3159 (kernel_close per block), OutputStream.hpp:
190-240 (the stitched stream), :225-239 (the in-order stitch the gather
replaces), InputStream.hpp:36-159 (the decoder the device path replaces)."""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from conftest import have_gpu

import bz2mi
from bz2mi import shard, synth

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not have_gpu(), reason="needs a HIP device")]


def _threads() -> int:
    return max(1, min(16, len(os.sched_getaffinity(0))))


def c4_stream(n: int, seg: int = 64 << 20) -> np.ndarray:
    """synth.mixed_bytes(n) (C4: 64 MiB segments of random / text / runs /
    ACGT, seed 0x5EED0003) with the segments generated on a thread pool."""
    out = np.empty(n, dtype=np.uint8)
    starts = list(range(0, n, seg))

    def fill(k):
        a = starts[k]
        m = min(seg, n - a)
        out[a:a + m] = synth.mixed_segment(k, m, synth.SEED_MIXED)

    with ThreadPoolExecutor(_threads()) as ex:
        list(ex.map(fill, range(len(starts))))
    return out


@pytest.mark.timeout(600)
def test_c4_8gib_units_equal_single_stream():
    """Config C4 at its full size on one MI355X: the 8 GiB mixed stream cut into
    8 units of 1 GiB (each with its tail halo, as ranks hold them), compressed
    with the unit protocol (chain token, seed-sum exchange, bit offsets, CRC
    shares), settled and gathered in order into one stream -- the same bytes
    as one compress_device call over the whole input, decoding back to the
    input on the device."""
    n = 8 << 30
    K = 8
    U = n // K
    level, p = 9, 10
    dev = torch.device("cuda", 0)
    host = c4_stream(n)
    assert np.array_equal(host[:1 << 20], synth.mixed_bytes(1 << 20))  # the C4 generator's bytes
    x = torch.from_numpy(host).to(dev)
    del host
    # one device call over the whole stream
    cap = bz2mi.compress_bound(n, level, 10000)
    whole = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx = bz2mi.Context(level, p, 10000)
    m = ctx.compress_device(x.data_ptr(), n, whole.data_ptr(), cap)
    ctx.close()
    whole = whole[:m].clone()
    torch.cuda.empty_cache()
    # the same stream in 8 units (world 1: every unit on this rank)
    ctx = bz2mi.Context(level, p, 10000)
    halo = bz2mi.unit_halo(level, 10000)
    owners = [0] * K
    units = {}
    for g in range(K):
        a, b = g * U, (g + 1) * U
        end = min(n, b + halo)
        u = shard.DeviceUnit(ctx, dev)
        u.begin(x[a:end].clone(), b - a, end - b, end == n)
        units[g] = u
    lay = shard.compress_units(units, owners, p, level)
    assert sum(lay.nblocks) > 8 and all(nb > 0 for nb in lay.nblocks)
    assert any(lay.offsets[g] & 7 for g in range(1, K)), "units should start mid-byte"
    out = torch.zeros(lay.stream_bytes + 64, dtype=torch.uint8, device=dev)
    got = shard.gather_stream_device(lay, shard.settle(lay), out, level)
    assert got.numel() == m
    assert torch.equal(got, whole)
    del units, lay, out, got, u
    ctx.close()
    torch.cuda.empty_cache()
    # and back on the device
    y = torch.empty(n, dtype=torch.uint8, device=dev)
    d = bz2mi.Decompressor(10000)
    assert d.decompress_device(whole.data_ptr(), m, y.data_ptr(), n) == n
    assert torch.equal(x, y)


@pytest.mark.timeout(600)
def test_c3_text_1gib_matches_cpuref(cpuref):
    """Config C3 stand-in at its full size (enwik9 is not available offline):
    1 GiB of synth.text_bytes (seed 0x5EED0002, the bench's --data text input)
    compressed by compress_device at -9, p = 10 is the C restatement's stream
    (cpu_ref on the host's cores, pinned to O_ref) byte for byte -- the text
    BWT paths (pair path, wave-level partitions, LDS-text batch sorts, ties,
    doubling) at full size -- and decodes back on the device."""
    n = 1 << 30
    host = synth.text_bytes(n, synth.SEED_TEXT)
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(host).to(dev)
    cap = bz2mi.compress_bound(n, 9, 10000)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx = bz2mi.Context(9, 10, 10000)
    m = ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)
    stream = out[:m].cpu().numpy().tobytes()
    assert stream == cpuref.compress(host.tobytes(), 9, 10, threads=_threads())
    y = torch.empty(n, dtype=torch.uint8, device=dev)
    d = bz2mi.Decompressor(10000)
    assert d.decompress_device(out.data_ptr(), m, y.data_ptr(), n) == n
    assert torch.equal(x, y)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("unit", [10000, 100000])
def test_c3_realtext_1gib_matches_cpuref(cpuref, unit):
    """Config C3 at its full size with the enwik9-like text (synth.realtext_bytes,
    seed 0x5EED0004, the bench's --data realtext input: ~150 distinct bytes and
    ~2,200 byte pairs per 90 KB block, markup, UTF-8, repeated passages of
    0.2-20 KB): compress_device at -9, p = 10 equals the C restatement's stream
    byte for byte (the text BWT kernel for any alphabet, its deferred deep ties,
    the general path for the blocks it hands back), at the reference's block
    size and in the 900 KB mode, and decodes back on the device."""
    n = 1 << 30
    host = synth.realtext_bytes(n, synth.SEED_REALTEXT, threads=_threads())
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(host).to(dev)
    cap = bz2mi.compress_bound(n, 9, unit)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx = bz2mi.Context(9, 10, unit)
    m = ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)
    stream = out[:m].cpu().numpy().tobytes()
    assert stream == cpuref.compress(host.tobytes(), 9, 10, unit=unit, threads=_threads())
    del host
    y = torch.empty(n, dtype=torch.uint8, device=dev)
    d = bz2mi.Decompressor(unit)
    assert d.decompress_device(out.data_ptr(), m, y.data_ptr(), n) == n
    assert torch.equal(x, y)


def test_unit_assemble_waits_for_null_stream_users():
    """bz2mi_unit_assemble writes the caller's buffer only after the work queued
    on the caller's stream (NULL: the null stream) that still uses it: the
    buffer is being overwritten by queued kernels when assemble is called, with
    no synchronize in between."""
    dev = torch.device("cuda", 0)
    data = synth.mixed_bytes(24 << 20, segment=4 << 20)
    x = torch.from_numpy(data).to(dev)
    n = x.numel()
    ctx = bz2mi.Context(9, 10, 10000)
    cap = bz2mi.compress_bound(n, 9, 10000)
    ref = torch.empty(cap, dtype=torch.uint8, device=dev)
    m = ctx.compress_device(x.data_ptr(), n, ref.data_ptr(), cap)
    u = bz2mi.Unit(ctx)
    u.begin(x.data_ptr(), n, 0, shard.UNIT_ENDS_STREAM, 0)
    ex, nb = u.chain(0, 0)
    assert nb > 0
    u.sums()
    bits, crc = u.encode(np.zeros(10 * 258, dtype=np.uint32))
    buf = torch.empty(cap, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    for v in range(31):  # queued on the null stream, still running when assemble is called
        buf.fill_(v)
    nbytes = u.assemble(0, 0, shard.UNIT_FIRST | shard.UNIT_LAST, buf.data_ptr(), buf.numel(), 0)
    assert nbytes == m
    assert torch.equal(buf[:m], ref[:m])
    u.close()


@pytest.mark.timeout(600)
def test_c4_mixed_512mib_matches_cpuref(cpuref):
    """Config C4's data against the C restatement, not only against the
    device's own single call: the first 512 MiB of the C4 stream (eight 64 MiB
    segments of random, text, run-heavy and ACGT bytes) compressed by
    compress_device at -9, p = 10 and, cut into 4 stream units (the layout
    the 8-GPU configuration shards), by the unit protocol -- both equal to
    cpu_ref's stream (pinned to O_ref) byte for byte."""
    n = 512 << 20
    host = c4_stream(n)
    want = cpuref.compress(host.tobytes(), 9, 10, threads=_threads())
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(host).to(dev)
    cap = bz2mi.compress_bound(n, 9, 10000)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx = bz2mi.Context(9, 10, 10000)
    m = ctx.compress_device(x.data_ptr(), n, out.data_ptr(), cap)
    assert out[:m].cpu().numpy().tobytes() == want
    K, halo = 4, bz2mi.unit_halo(9, 10000)
    U = n // K
    units = {}
    for g in range(K):
        a, b = g * U, (g + 1) * U
        end = min(n, b + halo)
        u = shard.DeviceUnit(ctx, dev)
        u.begin(x[a:end].clone(), b - a, end - b, end == n)
        units[g] = u
    lay = shard.compress_units(units, [0] * K, 10, 9)
    o2 = torch.zeros(lay.stream_bytes + 64, dtype=torch.uint8, device=dev)
    got = shard.gather_stream_device(lay, shard.settle(lay), o2, 9)
    assert got.cpu().numpy().tobytes() == want
    for u in units.values():
        u.close()
    ctx.close()
