"""Test helper: parse a .bz2 stream into its per-block fields (bzip2 format as
the reference writes it: OutputStream.hpp:126-128/192-213, kernel.cpp:3099-3122
close_block -> origPtr, writeSymbolMap :2483-2511, writeSelectorsAndHuffmanTables
:2991-3041, writeBlockData :3043-3062; trailer OutputStream.hpp:163-176).

parse_stream(data) -> {"level", "blocks": [{"crc", "rand", "orig", "present",
"ntables", "selectors", "lengths", "symbols"}], "stream_crc"}; `symbols` are
the MTF/RLE2 symbols in the block's alphabet including the end-of-block symbol,
i.e. what the reference's MTFAndRLE2StageEncoder (kernel.cpp:2561-2649) emitted.
Independent of any compressor in this repository."""
from __future__ import annotations

import numpy as np


class _Bits:
    def __init__(self, data: bytes):
        self.b = bytes(data) + b"\0" * 8
        self.pos = 0

    def read(self, n: int) -> int:
        p = self.pos
        i = p >> 3
        w = int.from_bytes(self.b[i:i + 8], "big")
        self.pos = p + n
        return (w >> (64 - (p & 7) - n)) & ((1 << n) - 1)

    def peek(self, n: int) -> int:
        p = self.pos
        i = p >> 3
        w = int.from_bytes(self.b[i:i + 8], "big")
        return (w >> (64 - (p & 7) - n)) & ((1 << n) - 1)


def _table(lengths: list[int]):
    """Canonical decode table (codes by (length, symbol)) as a 2^M lookup."""
    M = max(lengths)
    sym = np.zeros(1 << M, dtype=np.int32)
    ln = np.zeros(1 << M, dtype=np.int32)
    code = 0
    for L in range(1, M + 1):
        for s, l in enumerate(lengths):
            if l == L:
                lo = code << (M - L)
                hi = (code + 1) << (M - L)
                sym[lo:hi] = s
                ln[lo:hi] = L
                code += 1
        code <<= 1
    return M, sym.tolist(), ln.tolist()


def parse_stream(data: bytes) -> dict:
    r = _Bits(data)
    if data[:3] != b"BZh":
        raise ValueError("not a bzip2 stream")
    r.pos = 24
    level = r.read(8) - 0x30
    blocks = []
    while True:
        magic = r.read(48)
        if magic == 0x177245385090:
            return {"level": level, "blocks": blocks, "stream_crc": r.read(32)}
        if magic != 0x314159265359:
            raise ValueError(f"bad block magic at bit {r.pos - 48}")
        crc = r.read(32)
        rand = r.read(1)
        orig = r.read(24)
        used = r.read(16)
        present = []
        for i in range(16):
            if used & (0x8000 >> i):
                m = r.read(16)
                present += [16 * i + j for j in range(16) if m & (0x8000 >> j)]
        alpha = len(present) + 2
        ntab = r.read(3)
        nsel = r.read(15)
        mtf = list(range(ntab))
        sels = []
        for _ in range(nsel):
            k = 0
            while r.read(1):
                k += 1
            v = mtf.pop(k)
            mtf.insert(0, v)
            sels.append(v)
        lengths = []
        for _ in range(ntab):
            cur = r.read(5)
            ls = []
            for _ in range(alpha):
                while r.read(1):
                    cur += -1 if r.read(1) else 1
                ls.append(cur)
            lengths.append(ls)
        tabs = [_table(ls) for ls in lengths]
        syms = []
        eob = alpha - 1
        g = 0
        while True:
            M, st, lt = tabs[sels[g // 50]] if g // 50 < len(sels) else tabs[0]
            v = r.peek(M)
            s = st[v]
            r.pos += lt[v]
            syms.append(s)
            g += 1
            if s == eob:
                break
        blocks.append({"crc": crc, "rand": rand, "orig": orig, "present": present, "ntables": ntab,
                       "selectors": sels, "lengths": lengths, "symbols": syms})
