"""One logical stream compressed in units: the unit
protocol of include/bz2mi.h driven by bz2mi.shard must give the bytes of the
single-device stream for the concatenated input (OutputStream.hpp:131-240).

CPU tests run the protocol on the C restatement's units (cpuref_unit_*) in one
process and across two gloo ranks; the `gpu` tests run the device units
(bz2mi_unit_*) in one process and in two processes sharing cuda:0."""
from __future__ import annotations

import bz2
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import CpuRef, CpuRefUnit, have_gpu, unit_buffers

import bz2mi
from bz2mi import shard, synth


def _stream_case(n: int, seed: int) -> bytes:
    """Mixed data with every boundary hazard: random, text, long runs (a 300 KB
    run spans several -1 blocks, runs of 4..300 cut RLE1 pieces), ACGT."""
    rng = np.random.Generator(np.random.PCG64(seed))
    parts = [synth.random_bytes(n // 5, seed), synth.text_bytes(n // 5, seed + 1),
             np.full(300_000, 0x41, dtype=np.uint8), synth.runs_bytes(n // 5, seed + 2),
             synth.small_alphabet_bytes(n // 5, seed + 3), np.full(777, 7, dtype=np.uint8),
             rng.integers(0, 256, size=n // 10, dtype=np.uint8)]
    return np.concatenate(parts).tobytes()


def _cuts(n: int, seed: int, k: int, S: int) -> list[int]:
    rng = np.random.Generator(np.random.PCG64(seed))
    cuts = sorted(set(int(v) for v in rng.integers(1, n - 1, size=k)))
    # a few adversarial ones: tiny units (inside one block), cuts inside the long run
    extra = [cuts[0] + 1, cuts[0] + 3, n // 5 * 2 + 100_000, n // 5 * 2 + 100_255, n - 2]
    return sorted(set(c for c in cuts + extra if 0 < c < n))


def run_units(data: bytes, cuts: list[int], level: int, p: int, unit: int = 10000) -> bytes:
    halo = bz2mi.unit_halo(level, unit)
    units = {}
    for g, (buf, n_own, n_halo, ends) in enumerate(unit_buffers(data, cuts, halo)):
        u = CpuRefUnit(level, p, unit)
        u.begin(buf, n_own, n_halo, ends)
        units[g] = u
    lay = shard.compress_units(units, [0] * len(units), p, level)
    return shard.gather_stream_host(lay, level)


@pytest.mark.parametrize("level,p", [(1, 10), (1, 3), (2, 1), (9, 10)])
def test_units_one_process_equal_single_stream(level, p):
    data = _stream_case(1_200_000, 0x5EED0101 + level)
    want = CpuRef().compress(data, level, p)
    got = run_units(data, _cuts(len(data), 7 * level + p, 6, level * 10000), level, p)
    assert got == want
    assert bz2.decompress(got) == data


def test_units_edge_layouts():
    data = _stream_case(400_000, 0x5EED0202)
    want = CpuRef().compress(data, 1, 10)
    for cuts in ([], [1], [len(data) - 1], list(range(1000, len(data), 37_000)),
                 [5, 6, 7, 8, 9, 10]):
        assert run_units(data, cuts, 1, 10) == want, cuts
    # the whole stream one long run: every unit but the first covered by others
    run = bytes(2_000_000)
    assert run_units(run, [100, 200_000, 1_000_000], 1, 10) == CpuRef().compress(run, 1, 10)
    # empty stream
    assert shard.empty_stream(9) == CpuRef().compress(b"", 9, 10)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class SpecProbeUnit(CpuRefUnit):
    """A CPU unit with a speculate() that only counts: drives the protocol's
    token wait (irecv, speculation while the token is out) on gloo ranks."""

    def speculate(self):
        self.spec_calls = getattr(self, "spec_calls", 0) + 1
        return 0


def _cpu_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = _stream_case(1_500_000, 0x5EED0303)
    cuts = _cuts(len(data), 11, 9, 10000)
    halo = bz2mi.unit_halo(1, 10000)
    bufs = unit_buffers(data, cuts, halo)
    owners = shard.interleaved_owners(len(bufs), world)
    units = {}
    for g, (buf, n_own, n_halo, ends) in enumerate(bufs):
        if owners[g] == rank:
            u = SpecProbeUnit(1, 10, 10000)
            u.begin(buf, n_own, n_halo, ends)
            units[g] = u
    lay = shard.compress_units(units, owners, 10, 1)
    got = shard.gather_stream_host(lay, 1)
    if rank == 0:
        q.put(got == CpuRef().compress(data, 1, 10))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_two_ranks_one_stream():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert ok
    assert all(p.exitcode == 0 for p in procs)


class TensorPieceUnit(CpuRefUnit):
    """A CPU unit whose assemble() returns its bytes as a (uint8 tensor, nbytes)
    piece with spare room after them, the shape DeviceUnit gives settle() and
    gather_stream_device() -- so the point-to-point gather runs on gloo ranks."""

    def assemble(self, bit_offset, crc_before, flags):
        b = super().assemble(bit_offset, crc_before, flags)
        t = torch.zeros(len(b) + 64, dtype=torch.uint8)
        t[: len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        return t, len(b)


def _p2p_worker(rank, world, port, q):
    """settle() + gather_stream_device() across gloo ranks: every unit's piece
    goes point-to-point (batch_isend_irecv) to rank 0, OR-merging the shared
    boundary bytes of units that start mid-byte (OutputStream.hpp:225-239)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = _stream_case(1_500_000, 0x5EED0505)
    cuts = _cuts(len(data), 13, 9, 10000)
    bufs = unit_buffers(data, cuts, bz2mi.unit_halo(1, 10000))
    owners = shard.interleaved_owners(len(bufs), world)
    units = {}
    for g, (buf, n_own, n_halo, ends) in enumerate(bufs):
        if owners[g] == rank:
            u = TensorPieceUnit(1, 10, 10000)
            u.begin(buf, n_own, n_halo, ends)
            units[g] = u
    lay = shard.compress_units(units, owners, 10, 1)
    mid = sum(1 for g in range(len(bufs)) if lay.nblocks[g] and g != lay.first and lay.offsets[g] & 7)
    settled = shard.settle(lay)
    out = torch.zeros(lay.stream_bytes + 16, dtype=torch.uint8) if rank == 0 else None
    got = shard.gather_stream_device(lay, settled, out, 1, dst=0)
    if rank == 0:
        q.put((bytes(got.numpy().tobytes()) == CpuRef().compress(data, 1, 10), mid,
               len({owners[g] for g in range(len(bufs)) if lay.nblocks[g]})))
    else:
        assert got is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_gloo_p2p_gather_one_stream(world):
    """The ordered point-to-point gather of bz2mi.shard (the RCCL path of config
    C4) on CPU tensors over gloo: both sides of batch_isend_irecv, units that
    start mid-byte, pieces on every rank -> the single-stream cpu_ref bytes."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_p2p_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok, mid, ranks = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert ok
    assert mid >= 3, "the layout must exercise mid-byte unit boundaries"
    assert ranks == world, "every rank must hold pieces"
    assert all(p.exitcode == 0 for p in procs)


# ---------------------------------------------------------------- device ----

def _device_units(ctx, data_t: torch.Tensor, cuts: list[int], owners, rank, level, unit=10000):
    halo = bz2mi.unit_halo(level, unit)
    n = data_t.numel()
    bounds = [0] + list(cuts) + [n]
    units = {}
    for g, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
        if owners[g] != rank:
            continue
        end = min(n, b + halo)
        buf = data_t[a:end].clone()  # a unit's own buffer (bytes + halo), as a rank would hold it
        u = shard.DeviceUnit(ctx, data_t.device)
        u.begin(buf, b - a, end - b, end == n)
        units[g] = u
    return units


@pytest.mark.gpu
@pytest.mark.skipif(not have_gpu(), reason="needs a HIP device")
@pytest.mark.parametrize("level,p,n", [(9, 10, 24 << 20), (1, 10, 3 << 20), (1, 3, 2 << 20)])
def test_device_units_equal_single_stream(level, p, n):
    data = _stream_case(n, 0x5EED0404 + level)
    dev = torch.device("cuda", 0)
    x = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    ctx = bz2mi.Context(level, p, 10000)
    cuts = _cuts(len(data), 3 + level, 5, level * 10000)
    owners = [0] * (len(cuts) + 1)
    units = _device_units(ctx, x, cuts, owners, 0, level)
    lay = shard.compress_units(units, owners, p, level)
    out = torch.empty(lay.stream_bytes + 64, dtype=torch.uint8, device=dev)
    got = shard.gather_stream_device(lay, shard.settle(lay), out, level).cpu().numpy().tobytes()
    cap = bz2mi.compress_bound(len(data), level, 10000)
    o2 = torch.empty(cap, dtype=torch.uint8, device=dev)
    m = ctx.compress_device(x.data_ptr(), len(data), o2.data_ptr(), cap)
    whole = o2[:m].cpu().numpy().tobytes()
    assert got == whole
    assert whole == CpuRef().compress(data, level, p)
    # in-place assembly (BZ2MI_UNIT_IN_PLACE): every unit written at its bit
    # offset into one stream buffer, the shared boundary words carried over
    units = _device_units(ctx, x, cuts, owners, 0, level)
    o3 = torch.full((cap,), 0xA5, dtype=torch.uint8, device=dev)
    lay3 = shard.compress_units(units, owners, p, level, out=o3)
    assert lay3.out is not None and not lay3.pieces
    assert shard.gather_stream_device(lay3, shard.settle(lay3), None, level).cpu().numpy().tobytes() == whole


def _gpu_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    data = synth.mixed_bytes(16 << 20, synth.SEED_MIXED, segment=1 << 20).tobytes()
    x = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    ctx = bz2mi.Context(9, 10, 10000)
    cuts = [(16 << 20) * k // 6 for k in range(1, 6)]
    owners = shard.interleaved_owners(len(cuts) + 1, world)
    units = _device_units(ctx, x, cuts, owners, rank, 9)
    lay = shard.compress_units(units, owners, 10, 9)
    # device pieces -> host bytes, gathered over gloo (both ranks share one GPU)
    for g in list(lay.pieces):
        t, nb = lay.pieces[g]
        lay.pieces[g] = t[:nb].cpu().numpy().tobytes()
    got = shard.gather_stream_host(lay, 9)
    if rank == 0:
        q.put((got == bz2mi.compress(data, 9, 10), got == CpuRef().compress(data, 9, 10),
               bz2.decompress(got) == data))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.skipif(not have_gpu(), reason="needs a HIP device")
@pytest.mark.timeout(600)
def test_device_two_ranks_one_stream():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=500)
    for p in procs:
        p.join(timeout=60)
    assert res == (True, True, True)
    assert all(p.exitcode == 0 for p in procs)


# ------------------------------------------------------- speculation ----

def _split_starts(data: bytes, S: int) -> list[int]:
    """Block starts of the RLE1 split of `data` (the C restatement)."""
    L = CpuRef().L
    mx = len(data) // (S - 6) * 2 + 16
    st = (ctypes.c_uint64 * mx)()
    nb = L.cpuref_split(data, len(data), S, None, 0, st, None, None, mx)
    assert nb > 0
    return list(st[:nb])


def _spec_case():
    """A stream and cuts for speculation (bz2mi_unit_speculate): a chain's
    offset is kept block after block in RLE1-output units, so two chains meet
    only where a few bytes of offset vanish in 5-byte run flushes -- here a
    region of runs of 4.  Units: entry 1 and 3 bytes into the unit just before
    such flushes (the chains merge), a cut on a block start (the speculation
    is the chain), cuts inside a long zero run (mid-run entries) and in
    random / text data (the speculation mispredicts and never merges)."""
    quad = np.repeat(np.tile(np.array([0x61, 0x62], dtype=np.uint8), 50_000), 4)
    parts = [synth.random_bytes(300_000, 41), quad, synth.runs_bytes(1_500_000, 42), synth.random_bytes(300_000, 43),
             np.zeros(800_000, dtype=np.uint8), synth.text_bytes(500_000, 44), synth.runs_bytes(1_000_000, 45)]
    data = np.concatenate(parts).tobytes()
    S = 10000
    allst = _split_starts(data, S)
    cuts = [[s for s in allst if s > 250_000][0] - 1, [s for s in allst if s > 1_000_000][0] - 3,
            [s for s in allst if s > 2_000_000][0], 2_900_000, 3_100_000, 3_700_000]
    halo = bz2mi.unit_halo(1, 10000)
    bounds = [0] + cuts + [len(data)]
    expect = []  # per unit: (true blocks, entry, index of the first start shared with the chain from byte 0)
    for a, b in zip(bounds[:-1], bounds[1:]):
        tr = [s - a for s in allst if a <= s < b]
        sp = set(s for s in _split_starts(data[a:min(len(data), b + halo)], S) if s < b - a)
        entry = min([s for s in allst if s >= a], default=len(data)) - a
        expect.append((len(tr), entry, next((i for i, s in enumerate(tr) if s in sp), None)))
    return data, cuts, expect


def test_spec_case_layout():
    """The speculation layout has what the device test needs (C restatement):
    merging units, an exact one and mispredicting ones."""
    _, cuts, expect = _spec_case()
    merging = [g for g, (nb, e, first) in enumerate(expect) if e > 0 and first is not None and first + 2 < nb]
    exact = [g for g, (nb, e, first) in enumerate(expect) if g > 0 and e == 0]
    never = [g for g, (nb, e, first) in enumerate(expect) if nb > 0 and first is None]
    assert merging and exact and len(never) >= 2, expect


def _spec_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    data, cuts, _ = _spec_case()
    x = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    ctx = bz2mi.Context(1, 10, 10000)
    owners = shard.interleaved_owners(len(cuts) + 1, world)
    units = _device_units(ctx, x, cuts, owners, rank, 1)
    lay = shard.compress_units(units, owners, 10, 1, speculate="always")
    info = {g: units[g].chain_info() for g in units}
    for g in list(lay.pieces):
        t, nb = lay.pieces[g]
        lay.pieces[g] = t[:nb].cpu().numpy().tobytes()
    got = shard.gather_stream_host(lay, 1)
    infos = [None] * world
    dist.all_gather_object(infos, info)
    if rank == 0:
        allinfo = {}
        for d in infos:
            allinfo.update(d)
        q.put((got == bz2mi.compress(data, 1, 10), got == CpuRef().compress(data, 1, 10), lay.nblocks, allinfo))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.skipif(not have_gpu(), reason="needs a HIP device")
@pytest.mark.timeout(600)
def test_device_two_ranks_speculation():
    """Two gloo ranks on cuda:0, every unit speculated: units cut mid-run and
    mid-block whose speculation mispredicts, merges or is exact -> the single
    stream, and the chain outcomes agree with the C restatement's chains."""
    _, _, expect = _spec_case()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_spec_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    same_gpu, same_ref, nblocks, info = q.get(timeout=500)
    for p in procs:
        p.join(timeout=60)
    assert same_gpu and same_ref
    assert all(p.exitcode == 0 for p in procs)
    merged = 0
    for g, (nb, entry, first) in enumerate(expect):
        assert nblocks[g] == nb, (g, nblocks[g], nb)
        if g == 0 or nb == 0:
            continue
        i = info[g]
        assert i["speculated"], (g, i)
        assert i["spliced"] + i["chained"] == nb, (g, i)
        if entry == 0:
            assert i["spliced"] == nb and i["chained"] == 0, (g, i)  # the speculation is the chain
        elif first is None:
            assert i["spliced"] == 0, (g, i)  # mispredicted: the chain from the entry runs in full
        else:
            # merged (checked once per chain round): chained at least up to the first shared start
            assert i["spliced"] == 0 or i["chained"] >= first, (g, i)
            merged += i["spliced"] > 0
    assert merged >= 1, info


def _seed_worker(rank, world, port, q, seeds):
    """The unit protocol on `world` gloo ranks with the seed sums exchanged by
    all-gather rounds (or the stream-order token), units cut mid-run and
    inside blocks; rank 0 reports equality with the single stream and every
    rank its host timeline (chain token arrivals, rounds, encodes)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = _stream_case(1_200_000, 0x5EED0606)
    cuts = _cuts(len(data), 17, 10, 10000)
    bufs = unit_buffers(data, cuts, bz2mi.unit_halo(1, 10000))
    owners = shard.interleaved_owners(len(bufs), world)
    units = {}
    for g, (buf, n_own, n_halo, ends) in enumerate(bufs):
        if owners[g] == rank:
            u = CpuRefUnit(1, 3, 10000)
            u.begin(buf, n_own, n_halo, ends)
            units[g] = u
    trace = []
    lay = shard.compress_units(units, owners, 3, 1, seeds=seeds, trace=trace)
    got = shard.gather_stream_host(lay, 1)
    rounds = sum(1 for e in trace if e[0] == "round")
    if rank == 0:
        q.put((got == CpuRef().compress(data, 1, 3), len(bufs), rounds,
               sum(1 for g in range(len(bufs)) if lay.nblocks[g] == 0)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("seeds", ["rounds", "token"])
def test_gloo_four_ranks_seed_exchange(seeds):
    """World 4: seed sums by one all-gather per round of units plus an
    exclusive scan in stream order (SURVEY 8(e) exchange 1), and the token
    alternative; p = 3 so every slot's running sum crosses ranks.  Equal to
    the single-stream cpu_ref bytes; the rounds path takes ceil(units / 4)
    collectives."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seed_worker, args=(r, world, port, q, seeds)) for r in range(world)]
    for p in procs:
        p.start()
    ok, nunits, rounds, empty = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert ok
    assert nunits >= 12 and empty >= 1, (nunits, empty)
    assert rounds == (-(-nunits // world) if seeds == "rounds" else 0)
    assert all(p.exitcode == 0 for p in procs)
