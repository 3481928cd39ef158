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


SEED_REALTEXT = 0x5EED0004

_PREFIXES = "un re in dis en non pre over mis sub inter fore de trans super semi anti mid under".split()
_ROOTS = (
    "act form port spect struct dict duct ject mit pos rupt scrib tract vert vis voc cred fer graph log "
    "phon photo chron bio geo therm hydr astr cycl dem gen man mar mort nat ped pend press sens sequ "
    "sign sol son tain temp ten terr tort var ven vid viv volv bank town river north south west east "
    "king church music film album war army league team season county village city road station school "
    "parish party court game book song band record ship island lake valley mount born died"
).split()
_SUFFIXES = ("s ed ing er ers ion ions ive ly ment ments ness able al ial ic ical ous ist ists ity ize "
             "ized ship ward wood ton ford ham burg land field").split()
_SEPS = ((b" ", 700), (b", ", 60), (b". ", 45), (b".\n", 18), (b"\n\n", 8), (b"; ", 6), (b": ", 6),
         (b" (", 9), (b") ", 9), (b" - ", 5), (b"'s ", 10), (b"\n* ", 8), (b"|", 10), (b" \"", 4), (b"\" ", 4),
         (b"-", 6), (b"\n", 10), (b"/", 3))
_MARKUP = (b"[[", b"]]", b"[[Category:", b"{{", b"}}", b"{{cite web |url=http://www.", b"|title=", b"|accessdate=",
           b"'''", b"''", b"\n== ", b" ==\n", b"\n=== ", b" ===\n", b"&quot;", b"&amp;", b"&lt;ref&gt;",
           b"&lt;/ref&gt;", b"&lt;br /&gt;", b"&nbsp;", b"http://www.", b".com/", b".org/wiki/", b"{{Infobox",
           b"\n| name = ", b"\n| image = ", b"\n| population = ", b"[[File:", b"|thumb|", b"px|", b"}}\n",
           b"{{reflist}}", b"ISBN ", b"{{convert|", b"|km|mi}}", b"<!-- ", b" -->", b"[[wikt:", b"#REDIRECT [[")


def _utf8_words(rng: np.random.Generator, count: int) -> list[bytes]:
    """Non-ASCII words (UTF-8): accented Latin, Cyrillic, Greek, CJK and Arabic."""
    words = []
    lat = "abcdefghiklmnoprstuvz"
    acc = "éèüöäñçåøáíóúâêßłšžć"
    for i in range(count):
        kind = i % 5
        m = int(rng.integers(2, 9))
        if kind == 0:  # accented Latin
            s = "".join(acc[int(rng.integers(len(acc)))] if rng.random() < 0.3 else lat[int(rng.integers(len(lat)))]
                        for _ in range(m + 2))
            s = s[0].upper() + s[1:] if rng.random() < 0.5 else s
        elif kind == 1:  # Cyrillic
            s = "".join(chr(0x430 + int(rng.integers(32))) for _ in range(m + 2))
        elif kind == 2:  # Greek
            s = "".join(chr(0x3B1 + int(rng.integers(24))) for _ in range(m + 1))
        elif kind == 3:  # CJK (a common-character range)
            s = "".join(chr(0x4E00 + int(rng.integers(2000))) for _ in range(1 + m // 3))
        else:  # Arabic
            s = "".join(chr(0x627 + int(rng.integers(36))) for _ in range(m))
        words.append(s.encode("utf-8"))
    return words


def _page_headers(rng: np.random.Generator, vocab: list[str], count: int) -> list[bytes]:
    """MediaWiki-export page headers (the boilerplate between enwik9's articles)."""
    out = []
    for i in range(count):
        title = " ".join(vocab[int(rng.integers(len(vocab)))].capitalize() for _ in range(int(rng.integers(1, 4))))
        pid = int(rng.integers(10, 3_000_000))
        rid = int(rng.integers(10_000, 50_000_000))
        ts = "%04d-%02d-%02dT%02d:%02d:%02dZ" % (2001 + int(rng.integers(6)), 1 + int(rng.integers(12)),
                                                 1 + int(rng.integers(28)), int(rng.integers(24)),
                                                 int(rng.integers(60)), int(rng.integers(60)))
        who = ("        <username>%s</username>\n        <id>%d</id>\n" %
               (vocab[int(rng.integers(len(vocab)))].capitalize() + str(int(rng.integers(100))), int(rng.integers(1, 900000)))
               if rng.random() < 0.8 else "        <ip>%d.%d.%d.%d</ip>\n" % tuple(int(v) for v in rng.integers(1, 255, 4)))
        comment = ("      <comment>%s</comment>\n" % " ".join(vocab[int(rng.integers(len(vocab)))] for _ in range(
            int(rng.integers(1, 7))))) if rng.random() < 0.6 else ""
        s = ("\n  </page>\n  <page>\n    <title>%s</title>\n    <id>%d</id>\n    <revision>\n      <id>%d</id>\n"
             "      <timestamp>%s</timestamp>\n      <contributor>\n%s      </contributor>\n%s"
             "      <text xml:space=\"preserve\">" % (title, pid, rid, ts, who, comment))
        out.append(s.encode())
    return out


_RT_TABLES: dict = {}


def _realtext_tables(seed: int):
    """The token table of realtext_bytes (built once per seed)."""
    if seed in _RT_TABLES:
        return _RT_TABLES[seed]
    rng = np.random.Generator(np.random.PCG64(seed))
    vocab = list(_SYLLABLES)
    for _ in range(9000):
        w = _ROOTS[int(rng.integers(len(_ROOTS)))]
        if rng.random() < 0.35:
            w = _PREFIXES[int(rng.integers(len(_PREFIXES)))] + w
        if rng.random() < 0.6:
            w = w + _SUFFIXES[int(rng.integers(len(_SUFFIXES)))]
        if rng.random() < 0.25:
            w = w + _SYLLABLES[int(rng.integers(len(_SYLLABLES)))]
        vocab.append(w)
    V = len(vocab)
    # token table: words in three cases, numbers, UTF-8 words, markup, page headers, separators
    words = [w.encode() for w in vocab]
    title = [w.capitalize().encode() for w in vocab]
    upper = [w.upper().encode() for w in vocab]
    nums = []
    for i in range(4000):
        k = i % 6
        if k == 0:
            nums.append(str(1700 + int(rng.integers(325))))
        elif k == 1:
            nums.append(str(int(rng.integers(1, 100))))
        elif k == 2:
            nums.append("{:,}".format(int(rng.integers(1000, 10_000_000))))
        elif k == 3:
            nums.append("%d.%d" % (int(rng.integers(100)), int(rng.integers(100))))
        elif k == 4:
            nums.append("%04d-%02d-%02d" % (1900 + int(rng.integers(120)), 1 + int(rng.integers(12)),
                                            1 + int(rng.integers(28))))
        else:
            nums.append(str(int(rng.integers(100, 100000))))
    nums_b = [s.encode() for s in nums]
    utf = _utf8_words(rng, 600)
    heads = _page_headers(rng, vocab, 3000)
    seps = [s for s, _ in _SEPS]
    toks = words + title + upper + nums_b + utf + list(_MARKUP) + heads + seps
    off = {"title": V, "upper": 2 * V, "num": 3 * V}
    off["utf"] = off["num"] + len(nums_b)
    off["mark"] = off["utf"] + len(utf)
    off["head"] = off["mark"] + len(_MARKUP)
    off["sep"] = off["head"] + len(heads)
    cnt = {"num": len(nums_b), "utf": len(utf), "mark": len(_MARKUP), "head": len(heads), "sep": len(seps)}
    flat = np.frombuffer(b"".join(toks), dtype=np.uint8)
    tlen = np.array([len(t) for t in toks], dtype=np.int64)
    tstart = np.concatenate([[0], np.cumsum(tlen)[:-1]])
    pw = np.cumsum(1.0 / np.arange(1, V + 1, dtype=np.float64) ** 1.05)
    pw /= pw[-1]
    sw = np.cumsum(np.array([w for _, w in _SEPS], dtype=np.float64))
    sw /= sw[-1]
    _RT_TABLES[seed] = (V, off, cnt, flat, tlen, tstart, pw, sw)
    return _RT_TABLES[seed]


REALTEXT_SEGMENT = 32 << 20


def realtext_segment(i: int, m: int, seed: int = SEED_REALTEXT) -> np.ndarray:
    """Segment i (m <= REALTEXT_SEGMENT bytes) of the realtext_bytes stream."""
    V, off, cnt, flat, tlen, tstart, pw, sw = _realtext_tables(seed)
    rng = np.random.Generator(np.random.PCG64([seed, i]))
    out = np.empty(m, dtype=np.uint8)
    pos = 0
    while pos < m:
        count = max(4096, (m - pos) // 10 + 64)
        w = np.searchsorted(pw, rng.random(count))
        j = rng.integers(0, 8, size=count)
        w2 = (np.roll(w, 2) * 31 + np.roll(w, 1) * 7 + j) % V  # order-2 flavour: phrases recur
        w = np.where(j < 3, w2, w)
        cls = rng.random(count)
        pick = rng.random(count)
        tok = w
        tok = np.where(cls < 0.10, w + off["title"], tok)
        tok = np.where((cls >= 0.10) & (cls < 0.105), w + off["upper"], tok)
        for name, lo, hi in (("num", 0.105, 0.155), ("utf", 0.155, 0.17), ("mark", 0.17, 0.245),
                             ("head", 1.0 - 1.0 / 1400, 1.0)):
            tok = np.where((cls >= lo) & (cls < hi), off[name] + (pick * cnt[name]).astype(np.int64), tok)
        sep = off["sep"] + np.searchsorted(sw, rng.random(count))
        seq = np.empty(2 * count, dtype=np.int64)
        seq[0::2] = tok
        seq[1::2] = sep
        L = tlen[seq]
        ends = np.cumsum(L)
        total = int(ends[-1])
        idx = np.repeat(tstart[seq] - (ends - L), L) + np.arange(total)
        k = min(total, m - pos)
        out[pos:pos + k] = flat[idx[:k]]
        pos += k
    # repeated passages: ~7 % of the bytes are copies of 0.2-20 KB from 1 KB to 8 MB back
    nrep = int(m * 0.07 / 3000) + 1
    dst = np.sort(rng.integers(0, m, size=nrep))
    ln = np.exp(rng.uniform(np.log(200), np.log(20000), size=nrep)).astype(np.int64)
    back = np.exp(rng.uniform(np.log(1024), np.log(8 << 20), size=nrep)).astype(np.int64)
    for d, L, bk in zip(dst.tolist(), ln.tolist(), back.tolist()):
        bk = max(bk, L)
        if d - bk < 0:
            continue
        L = min(L, m - d)
        out[d:d + L] = out[d - bk:d - bk + L]
    return out


def realtext_bytes(n: int, seed: int = SEED_REALTEXT, threads: int = 1) -> np.ndarray:
    """C3, enwik9-like (enwik9 itself is not available offline): English-like
    word text with mixed case, numbers and dates, punctuation, MediaWiki/XML
    markup and page headers, UTF-8 words (accented Latin, Cyrillic, Greek, CJK,
    Arabic) and repeated passages of 0.2-20 KB copied from 1 KB to 8 MB earlier
    -- ~150 distinct byte values and ~2,200 distinct byte pairs per 90 KB
    block (text_bytes has 27 bytes), bzip2 ratio ~0.28.  Made of 32 MiB
    segments with seeds of their own, so a prefix is the same stream and the
    segments can be generated on several threads."""
    out = np.empty(n, dtype=np.uint8)
    starts = list(range(0, n, REALTEXT_SEGMENT))
    _realtext_tables(seed)

    def fill(k):
        a = starts[k]
        e = min(n, a + REALTEXT_SEGMENT)
        out[a:e] = realtext_segment(k, e - a, seed)

    if threads > 1 and len(starts) > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(fill, range(len(starts))))
    else:
        for k in range(len(starts)):
            fill(k)
    return out


def repeats_bytes(n: int, seed: int = 0x5EED0077) -> np.ndarray:
    """realtext with long exact repeats inside every 90 KB block (a stress
    input for deep ties): a 30 KB passage copied 40 KB on, a 1 KB snippet
    repeated 20 times back to back (tandem: groups of ~20 rotations tied for
    up to 19 KB) and, every 180 KB, a 600-byte passage in three copies."""
    x = realtext_bytes(n, seed).copy()
    for o in range(0, n - 91000, 90000):
        x[o + 40000:o + 70000] = x[o:o + 30000]
        x[o + 71000:o + 91000] = np.tile(x[o + 5000:o + 6000], 20)
    for o in range(45000, n - 3000, 180000):
        x[o + 1000:o + 1600] = x[o:o + 600]
        x[o + 2000:o + 2600] = x[o:o + 600]
    return x


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
