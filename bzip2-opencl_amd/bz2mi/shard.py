"""One logical .bz2 stream, blocks sharded across ranks.

The reference compresses one stream on one device; what couples its blocks
is (OutputStream.hpp:131-240, kernel.cpp:3124-3159):
  * the block split: a chain through the RLE1 byte stream (a block ends once
    S-6 RLE1 bytes are flushed, OutputStream.hpp:179-188);
  * the per-slot frequency array that is never cleared (OutputStream.hpp:93,
    kernel.cpp:3155): block b seeds its Huffman tables from the
    sum of the histograms of every earlier block with the same b mod p;
  * the stream layout: blocks are bit-concatenated and the stream CRC chained
    in block order (OutputStream.hpp:190-240, :202).

Here the stream is cut into units (contiguous byte ranges; unit g on rank
owners[g], interleaved so that every rank gets work early) and each rank
compresses its units with the unit protocol of include/bz2mi.h:
  1. chain   -- the entry of unit g is the exit of unit g-1: one 16-byte token
                (entry, first block index) per unit, passed in stream order;
                a rank's blocks start compressing as soon as its chain is done
                while the token travels on.  While a rank waits for a token it
                speculates (bz2mi_unit_speculate): it chains the unit from its
                own first byte, and the chain from the real entry then runs
                only until it meets a speculative block start (a block's end
                depends only on the bytes from its start on);
  2. sums    -- the running sum of the per-unit slot sums (p x 258 uint32)
                passed in stream order like the chain token: the carried
                seeds of unit g are the sum over the units before it, and a
                unit is encoded (Huffman) as soon as they arrive, overlapping
                the later units' BWT / MTF;
  3. encode  -- all-gather of (bits, CRC share, blocks) per unit; exclusive scan
                of the bits gives each unit's stream bit offset, the CRC shares
                combine as crc' = rotl(crc, m) ^ share;
  4. assemble -- every unit lays out its bytes at its offset (first byte's top
                bit_offset&7 bits zero); gather_stream() collects them in order
                on one rank (RCCL point-to-point over xGMI for device pieces),
                OR-merging the shared boundary bytes.
Control messages go over a gloo group (host memory, tens of bytes each); the
only bulk transfer is the final gather.  The result equals the stream one
device produces for the concatenated input, byte for byte.

A unit object provides: chain(entry, first_block) -> (exit, nblocks),
optionally speculate() (before chain);
sums() -> uint32[p*258]; encode(carried) -> (bits, crc);
assemble(bit_offset, crc_before, flags) -> piece.  Device units are
bz2mi.Unit (DeviceUnit below); the tests drive the same protocol with the C
restatement's units.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

UNIT_ENDS_STREAM = 1
UNIT_FIRST = 1
UNIT_LAST = 2
UNIT_IN_PLACE = 4
MIDRUN = 1 << 63

EMPTY_STREAM_TAIL = bytes([0x17, 0x72, 0x45, 0x38, 0x50, 0x90, 0, 0, 0, 0])


def interleaved_owners(total_units: int, world: int) -> list[int]:
    """Unit g on rank g mod world: the chain token reaches every rank after one
    unit per rank, so no rank waits for a whole rank's worth of chain."""
    return [g % world for g in range(total_units)]


def _rotl(x: int, r: int) -> int:
    r &= 31
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF if r else x


@dataclass
class Layout:
    """Where every unit of the stream lands (known to all ranks after step 3)."""
    nblocks: list[int]
    bits: list[int]
    offsets: list[int]          # stream bit offset of each unit (units without blocks: -1)
    crc_before: list[int]
    first: int                  # unit that carries the stream header
    last: int                   # unit that carries the trailer
    stream_bits: int
    stream_crc: int
    owners: list = field(default_factory=list)
    empty: bool = False
    pieces: dict = field(default_factory=dict)   # local unit g -> piece (assemble output)
    out: object = None          # one rank, in-place assembly: the stream buffer holding every unit

    @property
    def stream_bytes(self) -> int:
        return (self.stream_bits + 7) // 8

    def byte_offset(self, g: int) -> int:
        return self.offsets[g] // 8


def _group_size(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _group_rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def _all_gather_rows(rows: np.ndarray, counts: list[int], group) -> list[np.ndarray]:
    """All-gather a [k_local, w] int64 table from every rank (k varies per
    rank; counts[r] known to all): returns the per-rank tables."""
    world = _group_size(group)
    if world == 1:
        return [rows]
    kmax = max(counts) if counts else 0
    w = rows.shape[1]
    buf = torch.zeros((max(kmax, 1), w), dtype=torch.int64)
    if rows.shape[0]:
        buf[: rows.shape[0]] = torch.from_numpy(rows.astype(np.int64))
    parts = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return [parts[r][: counts[r]].numpy() for r in range(world)]


def _seed_rounds(units: dict, owners: list[int], mine: list[int], w: int, group, encode,
                 trace: list | None = None) -> None:
    """Carried seeds by all-gathers (exchange 1): round j
    all-gathers the slot sums of every rank's j-th unit (global index + p x 258
    uint32), and an exclusive scan in stream order over the sums known so far
    gives the carried seeds of every unit whose predecessors are all known;
    this rank's such units are encoded right after the round.  With
    interleaved owners round j completes units [j N, (j+1) N), so a stream of
    N x k units takes k collectives instead of N k serial token hops, and
    every unit is still encoded as soon as its round is in."""
    world = _group_size(group)
    total = len(owners)
    rounds = max(sum(1 for o in owners if o == r) for r in range(world))
    known = {}
    carried_of = {}
    acc = np.zeros(w, dtype=np.uint32)
    k = 0                      # acc = uint32 sum of the sums of units < k
    todo = list(mine)
    for j in range(rounds):
        row = torch.zeros(w + 1, dtype=torch.int64)
        row[0] = -1
        if j < len(mine):
            g = mine[j]
            row[0] = g
            row[1:] = torch.from_numpy(units[g].sums().astype(np.uint32).astype(np.int64))
        parts = [torch.zeros_like(row) for _ in range(world)]
        dist.all_gather(parts, row, group=group)
        if trace is not None:
            trace.append(("round", j, time.perf_counter()))
        for t in parts:
            if int(t[0]) >= 0:
                known[int(t[0])] = t[1:].numpy().astype(np.uint32)
        while k < total and k in known:
            carried_of[k] = acc.copy()
            acc = acc + known.pop(k)   # uint32 wrap-around, as the reference's int array
            k += 1
        while todo and todo[0] in carried_of:
            g = todo.pop(0)
            encode(g, carried_of.pop(g))
    assert not todo, "seed rounds left units unencoded"


def compress_units(units: dict, owners: list[int], parallel: int, level: int, group=None,
                   speculate: str = "wait", out=None, seeds: str = "rounds", trace: list | None = None) -> Layout:
    """Run the unit protocol for this rank's units (dict global index -> unit,
    every unit already begun) of a stream of len(owners) units.  Returns the
    layout with this rank's assembled pieces.  speculate: "wait" (units whose
    token comes from another rank, while it is on its way), "always" (every
    unit but the first, before its chain: tests) or "never".  out (one rank,
    units with assemble_into): the stream buffer; every unit is assembled in
    place at its bit offset (no pieces, no gather copies).  seeds (world > 1):
    "rounds" (all-gather per round of units, _seed_rounds) or "token" (the
    running sum passed unit to unit in stream order).  trace: a list that
    gets (event, unit, time.perf_counter()) for the chain token's arrival
    ("recv"), every chain's end ("chain"), the seed rounds ("round") and every
    encode's end ("encode") -- the host timeline of the critical path."""
    clock = time.perf_counter
    rec = trace.append if trace is not None else (lambda e: None)
    me = _group_rank(group)
    total = len(owners)
    mine = sorted(units)
    assert all(owners[g] == me for g in mine), "units must belong to this rank"
    # 1. the chain, in stream order: token (entry, first block index)
    token = None
    nblocks_local = {}
    # units whose token comes from another rank: speculated while it travels
    waits = [g for g in mine if g > 0 and owners[g - 1] != me and hasattr(units[g], "speculate")]
    if speculate == "never":
        waits = []
    speculated = set()
    for g in mine:
        if speculate == "always" and g > 0 and hasattr(units[g], "speculate"):
            units[g].speculate()
            speculated.add(g)
        if g == 0:
            entry, first = 0, 0
        elif owners[g - 1] == me:
            entry, first = token
        else:
            t = torch.zeros(2, dtype=torch.int64)
            w = dist.irecv(t, src=owners[g - 1], group=group, tag=g)
            # this unit first, then the later ones, as long as the token is out
            for h in waits:
                if h < g or h in speculated:
                    continue
                if w.is_completed():
                    break
                units[h].speculate()
                speculated.add(h)
            w.wait()
            rec(("recv", g, clock()))
            entry, first = int(t[0]) & 0xFFFFFFFFFFFFFFFF, int(t[1])
        ex, nb = units[g].chain(entry, first)
        rec(("chain", g, clock()))
        nblocks_local[g] = nb
        token = (ex, first + nb)
        if g + 1 < total and owners[g + 1] != me:
            exs = ex - (1 << 64) if ex >= (1 << 63) else ex  # int64 bit pattern
            dist.send(torch.tensor([exs, first + nb], dtype=torch.int64), dst=owners[g + 1], group=group, tag=g + 1)
    # 2. slot sums -> carried seeds, passed in stream order like the chain
    # token (unit g's seeds are the uint32 sum of the slot sums of every unit
    # before it): a unit is encoded as soon as its own sums and the running
    # sum are known, so its Huffman coding overlaps the later units' BWT / MTF
    # instead of waiting for every unit of the stream
    w = parallel * 258
    acc = None
    rows = np.zeros((len(mine), 3), dtype=np.int64)
    local = _group_size(group) == 1
    in_place = local and out is not None and all(hasattr(units[g], "assemble_into") for g in mine)
    if local:  # one rank: offsets are known unit by unit too, so it assembles as it goes
        wb_all = [g for g in range(total) if nblocks_local[g] > 0]
        first_u = wb_all[0] if wb_all else -1
        last_u = wb_all[-1] if wb_all else -1
        G = C = 0
        offs_l = [-1] * total
        crcb_l = [0] * total
        pieces = {}
    if not local and seeds == "rounds":
        idx = {g: i for i, g in enumerate(mine)}

        def _enc(g, carried):
            bits, crc = units[g].encode(carried)
            rows[idx[g]] = (bits, crc & 0xFFFFFFFF, nblocks_local[g])
            rec(("encode", g, clock()))

        _seed_rounds(units, owners, mine, w, group, _enc, trace)
    for i, g in enumerate(mine if (local or seeds != "rounds") else []):
        if g == 0:
            acc = np.zeros(w, dtype=np.uint32)
        elif owners[g - 1] != me:
            t = torch.zeros(w, dtype=torch.int32)
            dist.recv(t, src=owners[g - 1], group=group, tag=total + 1 + g)
            rec(("sums", g, clock()))
            acc = t.numpy().view(np.uint32).copy()
        carried = acc.copy()
        acc = acc + units[g].sums().astype(np.uint32)   # uint32 wrap-around, as the reference's int array
        if g + 1 < total and owners[g + 1] != me:
            dist.send(torch.from_numpy(acc.view(np.int32).copy()), dst=owners[g + 1], group=group, tag=total + 2 + g)
        bits, crc = units[g].encode(carried)
        rec(("encode", g, clock()))
        rows[i] = (bits, crc & 0xFFFFFFFF, nblocks_local[g])
        if local and nblocks_local[g] > 0:
            offs_l[g], crcb_l[g] = G, C
            flags = (UNIT_FIRST if g == first_u else 0) | (UNIT_LAST if g == last_u else 0)
            if in_place:
                units[g].assemble_into(out, G, C, flags)
            else:
                pieces[g] = units[g].assemble(G, C, flags)
            G += bits + (32 if g == first_u else 0)
            C = _rotl(C, nblocks_local[g]) ^ (crc & 0xFFFFFFFF)
    if local:
        nbl = [nblocks_local[g] for g in range(total)]
        bl = [int(rows[i][0]) for i in range(total)]
        if first_u < 0:
            return Layout(nbl, bl, [-1] * total, [0] * total, -1, -1, 14 * 8, 0, list(owners), empty=True)
        lay = Layout(nbl, bl, offs_l, crcb_l, first_u, last_u, G + 80, C, list(owners))
        lay.pieces = pieces
        if in_place:
            lay.out = out
        return lay
    # 3. encode results -> bits, CRC share, blocks
    counts = [sum(1 for o in owners if o == r) for r in range(_group_size(group))]
    by_rank = [[g for g in range(total) if owners[g] == r] for r in range(len(counts))]
    tabs = _all_gather_rows(rows, counts, group)
    nbl = [0] * total
    bl = [0] * total
    cr = [0] * total
    for r, tab in enumerate(tabs):
        for i, g in enumerate(by_rank[r]):
            bl[g], cr[g], nbl[g] = int(tab[i][0]), int(tab[i][1]) & 0xFFFFFFFF, int(tab[i][2])
    with_blocks = [g for g in range(total) if nbl[g] > 0]
    if not with_blocks:
        return Layout(nbl, bl, [-1] * total, [0] * total, -1, -1, 14 * 8, 0, list(owners), empty=True)
    first_u, last_u = with_blocks[0], with_blocks[-1]
    offs = [-1] * total
    crcb = [0] * total
    G, C = 0, 0
    for g in with_blocks:
        offs[g] = G
        crcb[g] = C
        G += bl[g] + (32 if g == first_u else 0)
        C = _rotl(C, nbl[g]) ^ cr[g]
    lay = Layout(nbl, bl, offs, crcb, first_u, last_u, G + 80, C, list(owners))
    # 4. assemble this rank's pieces
    for g in mine:
        if nbl[g] == 0:
            continue
        flags = (UNIT_FIRST if g == first_u else 0) | (UNIT_LAST if g == last_u else 0)
        lay.pieces[g] = units[g].assemble(offs[g], crcb[g], flags)
    return lay


def empty_stream(level: int) -> bytes:
    return b"BZh" + bytes([0x30 + level]) + EMPTY_STREAM_TAIL


def merge_pieces(lay: Layout, pieces: dict, level: int) -> bytes:
    """Host-side merge of (global unit -> bytes) pieces into the stream."""
    if lay.empty:
        return empty_stream(level)
    out = bytearray(lay.stream_bytes)
    for g in sorted(pieces):
        b = pieces[g]
        o = lay.byte_offset(g)
        if len(b) == 0:
            continue
        out[o] |= b[0]
        out[o + 1: o + len(b)] = b[1:]
    return bytes(out)


def gather_stream_host(lay: Layout, level: int, dst: int = 0, group=None) -> bytes | None:
    """Ordered gather of host-byte pieces (gloo): the stream on `dst`."""
    world = _group_size(group)
    mine = {g: bytes(p) for g, p in lay.pieces.items()}
    if world == 1:
        return merge_pieces(lay, mine, level)
    got = [None] * world
    dist.all_gather_object(got, mine, group=group)
    if _group_rank(group) != dst:
        return None
    allp = {}
    for d in got:
        allp.update(d)
    return merge_pieces(lay, allp, level)


class DeviceUnit:
    """bz2mi.Unit with torch-allocated output: assemble() returns
    (uint8 device tensor, nbytes)."""

    def __init__(self, ctx, device: torch.device):
        import bz2mi
        self.unit = bz2mi.Unit(ctx)
        self.device = device
        self._out = None

    def begin(self, buf: torch.Tensor, n_own: int, n_halo: int, ends: bool, stream: int = 0):
        self.buf = buf  # keep the bytes alive until assembly
        self.unit.begin(buf.data_ptr(), n_own, n_halo, UNIT_ENDS_STREAM if ends else 0, stream)

    def speculate(self):
        return self.unit.speculate()

    def chain(self, entry, first_block):
        return self.unit.chain(entry, first_block)

    def chain_info(self):
        return self.unit.chain_info()

    def sums(self):
        return self.unit.sums()

    def encode(self, carried):
        self.bits, crc = self.unit.encode(carried)
        return self.bits, crc

    def assemble(self, bit_offset, crc_before, flags):
        need = (self.bits + 32 + 80 + 8) // 8 + 8
        need = (need + 255) // 256 * 256
        if self._out is None or self._out.numel() < need:
            self._out = torch.empty(int(need * 1.25) // 4 * 4 + 256, dtype=torch.uint8, device=self.device)
        # the buffer may still be read by work queued on torch's current stream
        # (a previous step's gather / copies): assembly waits for that stream
        stream = torch.cuda.current_stream(self.device).cuda_stream
        nbytes = self.unit.assemble(bit_offset, crc_before, flags, self._out.data_ptr(), self._out.numel(), stream)
        return self._out, nbytes

    def assemble_into(self, out: torch.Tensor, bit_offset, crc_before, flags):
        """In-place assembly into the stream buffer `out` (uint8 device
        tensor) at stream bit bit_offset; returns the stream bytes so far."""
        stream = torch.cuda.current_stream(self.device).cuda_stream
        return self.unit.assemble(bit_offset, crc_before, flags | UNIT_IN_PLACE, out.data_ptr(), out.numel(), stream)

    def timings(self):
        return self.unit.timings()

    def stats(self):
        return self.unit.stats()

    def close(self) -> None:
        self.unit.close()
        self._out = None


def settle(lay: Layout, ctl_group=None) -> dict:
    """Make this rank's device pieces disjoint: where a unit starts mid-byte,
    its first byte is OR-ed into the previous unit's last byte (one small
    all-gather over the control group), and the unit keeps the bytes after it.
    Returns {g: (tensor, lo, hi)}: stream bytes [lo, hi) are tensor[0:hi-lo]
    (a view); together the ranks' ranges tile the stream exactly."""
    if lay.out is not None:  # assembled in place: nothing to settle
        return {}
    world = _group_size(ctl_group)
    total = len(lay.nblocks)
    wb = [g for g in range(total) if lay.nblocks[g] > 0]
    prev = {b: a for a, b in zip(wb[:-1], wb[1:])}
    shared = {g for g in wb if g != lay.first and (lay.offsets[g] & 7) != 0}
    fb_local = {g: int(lay.pieces[g][0][0].item()) for g in lay.pieces if g in shared}
    if world > 1:
        got = [None] * world
        dist.all_gather_object(got, fb_local, group=ctl_group)
        fb = {}
        for d in got:
            fb.update(d)
    else:
        fb = fb_local
    nxt = {a: b for b, a in prev.items()}
    out = {}
    for g, (t, n) in lay.pieces.items():
        o = lay.byte_offset(g)
        lo, start = (o + 1, 1) if g in shared else (o, 0)
        if g in nxt and nxt[g] in shared:
            t[n - 1: n] |= fb[nxt[g]]
        out[g] = (t[start:n], lo, o + n)
    return out


def gather_stream_device(lay: Layout, settled: dict, out: torch.Tensor | None, level: int, dst: int = 0,
                         group=None):
    """Ordered gather of the settled device pieces onto `dst` into `out` (a
    uint8 device tensor of >= lay.stream_bytes on dst): every piece goes
    point-to-point (RCCL over xGMI) straight to its stream position."""
    me = _group_rank(group)
    world = _group_size(group)
    if lay.empty:
        if me != dst:
            return None
        e = empty_stream(level)
        out[: len(e)].copy_(torch.frombuffer(bytearray(e), dtype=torch.uint8))
        return out[: len(e)]
    if lay.out is not None:  # one rank, assembled in place
        if out is not None and out.data_ptr() != lay.out.data_ptr():
            out[: lay.stream_bytes].copy_(lay.out[: lay.stream_bytes])
            return out[: lay.stream_bytes]
        return lay.out[: lay.stream_bytes]
    total = len(lay.nblocks)
    # the byte ranges of every unit follow from the layout (known everywhere)
    wb = [g for g in range(total) if lay.nblocks[g] > 0]
    ranges = {}
    for i, g in enumerate(wb):
        o = lay.byte_offset(g)
        lo = o + 1 if (g != lay.first and (lay.offsets[g] & 7) != 0) else o
        hi = lay.byte_offset(wb[i + 1]) + (1 if (lay.offsets[wb[i + 1]] & 7) != 0 else 0) if i + 1 < len(wb) \
            else lay.stream_bytes
        ranges[g] = (lo, hi)
    ops = []
    for g in wb:
        lo, hi = ranges[g]
        if hi <= lo:
            continue
        if lay.owners[g] == me:
            t, lo2, hi2 = settled[g]
            assert (lo2, hi2) == (lo, hi), (g, lo, hi, lo2, hi2)
            if me == dst:
                out[lo:hi].copy_(t[: hi - lo])
            else:
                ops.append(dist.P2POp(dist.isend, t[: hi - lo], dst, group=group))
        elif me == dst:
            ops.append(dist.P2POp(dist.irecv, out[lo:hi], lay.owners[g], group=group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    if me != dst:
        return None
    return out[: lay.stream_bytes]
