"""Seeded synthetic byte streams for the parity tests and bench.py.

SURVEY.md section 8(d) names the workloads: C1 word-salad text, C2 random
bytes (seed 0x5EED0001), C3 English-like text (seed 0x5EED0002; enwik9 is not
available offline), C4 mixed-entropy stream (seed 0x5EED0003).  All generators
are deterministic numpy code so the same bytes can be produced on the host for
the oracle and on the GPU box for the device path.
"""
from __future__ import annotations

import numpy as np

SEED_RANDOM = 0x5EED0001
SEED_TEXT = 0x5EED0002
SEED_MIXED = 0x5EED0003

_SYLLABLES = (
    "the of and to in is was he for it with as his on be at by had are but "
    "from or have an they which one you were all we her she there would their "
    "will when who him been has more if no out so said what up its about into "
    "than them can only other time new some could these two may first then do "
    "any like my now over such our man me even most made after also did many "
    "off before must well back through years much where your way down should "
    "because each just those people how too little state good very make world "
    "still see own men work long here get both between life being under never "
    "day same another know while last might us great old year since against "
    "go came right used take three states himself few house use during without "
    "again place american around however home small found thought went say part "
    "once general high upon school every don does got united left number course "
    "war until always away something fact though water less public put think "
    "almost hand enough far took head yet government system better set told"
).split()


def random_bytes(n: int, seed: int = SEED_RANDOM) -> np.ndarray:
    """C2: uniformly random bytes."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.integers(0, 256, size=n, dtype=np.uint8)


def text_bytes(n: int, seed: int = SEED_TEXT) -> np.ndarray:
    """C1/C3: Zipf word salad with order-2 repeats, punctuation and line breaks
    (vectorised so a 1 GB sample is generated in seconds)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    vocab = list(_SYLLABLES)
    for i in range(1500):  # derived words: a Zipf-like, larger vocabulary
        a, b = rng.integers(0, len(_SYLLABLES), size=2)
        vocab.append(_SYLLABLES[a][: 1 + (i % 4)] + _SYLLABLES[b])
    seps = [b" "] * 37 + [b".\n", b", ", b"\n\n"]
    V = len(vocab)
    p = 1.0 / np.arange(1, V + 1, dtype=np.float64)
    p /= p.sum()
    # token table: every (word, separator) pair as one byte string
    toks = [w.encode() + sp for w in vocab for sp in (b" ", b".\n", b", ", b"\n\n")]
    flat = np.frombuffer(b"".join(toks), dtype=np.uint8)
    tlen = np.array([len(t) for t in toks], dtype=np.int64)
    tstart = np.concatenate([[0], np.cumsum(tlen)[:-1]])
    out = np.empty(n, dtype=np.uint8)
    pos = 0
    while pos < n:
        count = max(1024, (n - pos) // 6 + 64)
        w = rng.choice(V, size=count, p=p)
        j = rng.integers(0, 8, size=count)
        rep = j < 3  # order-2 flavour: a word determined by the previous two
        w2 = (np.roll(w, 2) * 31 + np.roll(w, 1) * 7 + j) % V
        w = np.where(rep, w2, w)
        pc = rng.integers(0, 40, size=count)
        sep = np.where(pc == 0, 1, np.where(pc == 1, 2, np.where(pc == 2, 3, 0)))
        tok = w * 4 + sep
        L = tlen[tok]
        ends = np.cumsum(L)
        total = int(ends[-1])
        idx = np.repeat(tstart[tok] - (ends - L), L) + np.arange(total)
        chunk = flat[idx]
        m = min(total, n - pos)
        out[pos:pos + m] = chunk[:m]
        pos += m
    return out


def runs_bytes(n: int, seed: int = SEED_MIXED, max_run: int = 300) -> np.ndarray:
    """Run-heavy bytes: random values repeated 1..max_run times (RLE1 stress)."""
    rng = np.random.Generator(np.random.PCG64(seed ^ 0x55))
    est = n // (max_run // 2) + 64
    out = []
    total = 0
    while total < n:
        vals = rng.integers(0, 256, size=est, dtype=np.uint8)
        lens = rng.integers(1, max_run + 1, size=est)
        chunk = np.repeat(vals, lens)
        out.append(chunk)
        total += chunk.size
    return np.concatenate(out)[:n]


def small_alphabet_bytes(n: int, seed: int = SEED_MIXED, k: int = 4) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed ^ 0xAA))
    alpha = np.frombuffer(b"ACGT"[:k] if k <= 4 else bytes(range(65, 65 + k)), dtype=np.uint8)
    return alpha[rng.integers(0, len(alpha), size=n)]


def mixed_segment(i: int, m: int, seed: int = SEED_MIXED) -> np.ndarray:
    """Segment i (m bytes) of the C4 stream: random, text, runs, ACGT in turn."""
    gens = [random_bytes, text_bytes, runs_bytes, small_alphabet_bytes]
    return gens[i % 4](m, seed + i)


def mixed_bytes(n: int, seed: int = SEED_MIXED, segment: int = 64 << 20, first_segment: int = 0) -> np.ndarray:
    """C4: rotate segments of random, text, run-heavy and small-alphabet data
    (the stream from segment `first_segment` on: any rank can make its part)."""
    out = np.empty(n, dtype=np.uint8)
    pos = 0
    i = first_segment
    while pos < n:
        m = min(segment, n - pos)
        out[pos:pos + m] = mixed_segment(i, m, seed)
        pos += m
        i += 1
    return out
