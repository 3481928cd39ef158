"""Device decompression (bz2mi_decompress*) on an MI355X.

Oracle: the original bytes.  Every stream decoded here was produced either by
O_ref (the reference's own compressor, committed fixtures), by bz2mi's
compressor (itself byte-identical to O_ref / cpu_ref, test_gpu.py) or by the
system bzip2 library (stock 900 KB blocks, unit 100000).  Error cases check
the reference decoder's messages (InputStream.hpp / BlockDecompressor.hpp).
"""
from __future__ import annotations

import bz2

import numpy as np
import pytest

from conftest import golden_file, golden_input

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bz():
    import bz2mi
    if bz2mi.lib().bz2mi_device_count() <= 0:
        pytest.fail("no HIP device: the gpu tests need an MI355X")
    return bz2mi


@pytest.fixture(scope="module")
def dec(bz):
    with bz.Decompressor(10000) as d:
        yield d


def test_golden_oref_streams(bz, dec, manifest):
    for name, e in sorted(manifest["cases"].items()):
        data = golden_input(name)
        for st in e["streams"]:
            assert dec.decompress(golden_file(st["file"])) == data, (name, st)


def _inputs():
    from bz2mi import synth
    yield "empty", b""
    yield "one", b"x"
    yield "text", synth.text_bytes(3 << 20).tobytes()
    yield "realtext", synth.realtext_bytes(3 << 20).tobytes()
    yield "repeats", synth.repeats_bytes(2 << 20).tobytes()
    yield "random", synth.random_bytes(3 << 20).tobytes()
    yield "runs", synth.runs_bytes(3 << 20).tobytes()
    yield "runs_long", synth.runs_bytes(2 << 20, max_run=5000).tobytes()
    yield "acgt", synth.small_alphabet_bytes(2 << 20).tobytes()
    yield "zeros", bytes(1 << 20)
    yield "periodic_ab", b"ab" * (1 << 18)
    yield "mixed", synth.mixed_bytes(4 << 20, segment=512 << 10).tobytes()


@pytest.mark.parametrize("level,p", [(9, 10), (1, 1)])
def test_round_trip_bz2mi_streams(bz, dec, level, p):
    for name, data in _inputs():
        z = bz.compress(data, level, p)
        assert dec.decompress(z) == data, (name, level, p)
        assert bz2.decompress(z) == data


def test_stock_bzip2_files_need_unit_100000(bz):
    from bz2mi import synth
    data = synth.text_bytes(3 << 20).tobytes() + synth.random_bytes(1 << 20).tobytes()
    z = bz2.compress(data, 9)
    with bz.Decompressor(100000) as d:
        assert d.decompress(z) == data
        assert d.decompress(bz2.compress(data[:12345], 1)) == data[:12345]
    # the reference's decoder limits blocks to digit x 10,000 bytes and 1801
    # selectors: a stock -9 file fails with "block Huffman tables invalid"
    # (the message its probe saw)
    with bz.Decompressor(10000) as d, pytest.raises(bz.DecompressError, match="block Huffman tables invalid"):
        d.decompress(z)


def test_decode_budget_smaller_than_the_stream(bz, monkeypatch):
    """A symbol budget (BZ2MI_DEC_BUDGET) far below the stream's decoded size:
    the stream is decoded in many windows with the same bytes (the
    budget bounds device memory whatever the input size)."""
    from bz2mi import synth
    data = synth.mixed_bytes(24 << 20, segment=2 << 20).tobytes()
    z = bz.compress(data, 9, 10)
    monkeypatch.setenv("BZ2MI_DEC_BUDGET", str(16 << 20))  # ~16 blocks per window of ~270
    with bz.Decompressor(10000) as d:
        assert d.decompress(z) == data


def test_900k_mode_round_trip(bz):
    from bz2mi import synth
    data = synth.mixed_bytes(5 << 20, segment=1 << 20).tobytes()
    z = bz.compress(data, 9, 10, unit=100000)
    with bz.Decompressor(100000) as d:
        assert d.decompress(z) == data


def test_concatenated_streams(bz, dec):
    a, b = b"first stream " * 1000, bytes(range(256)) * 700
    z = bz.compress(a, 9, 10) + bz.compress(b, 3, 2)
    # the reference's InputStream stops at the first end-of-stream marker
    assert dec.decompress(z) == a
    assert dec.decompress(z + b"\x00\x01") == a
    with bz.Decompressor(10000, concatenated=True) as d:
        assert d.decompress(z) == a + b
        # trailing bytes that start no stream are ignored (bzip2's behaviour)
        assert d.decompress(z + b"\x00\x01") == a + b


def _flip(z: bytes, byte: int, bit: int) -> bytes:
    b = bytearray(z)
    b[byte] ^= 1 << bit
    return bytes(b)


def test_errors_carry_the_reference_messages(bz, dec):
    from bz2mi import synth
    data = synth.text_bytes(400_000).tobytes()
    z = bz.compress(data, 9, 10)
    with pytest.raises(bz.DecompressError, match="Invalid BZip2 header"):
        dec.decompress(b"BZx9" + z[4:])
    with pytest.raises(bz.DecompressError, match="Invalid BZip2 header"):
        dec.decompress(b"BZh0" + z[4:])
    # stored block CRC of the first block: bits 80..111 of the stream
    with pytest.raises(bz.DecompressError, match="BZip2 block CRC error"):
        dec.decompress(_flip(z, 11, 3))
    # stored stream CRC: the last 32 bits before the padding
    with pytest.raises(bz.DecompressError, match="(BZip2 stream CRC error|BZip2 stream format error)"):
        dec.decompress(_flip(z, len(z) - 2, 0))
    with pytest.raises(bz.DecompressError):
        dec.decompress(z[: len(z) // 2])
    # corrupted Huffman data somewhere in the middle: some reference error
    with pytest.raises(bz.DecompressError):
        dec.decompress(_flip(z, len(z) // 3, 5))


def test_full_size_round_trip_on_device(bz):
    """256 MiB of mixed data: compress and decompress with device buffers."""
    import torch
    from bz2mi import synth
    n = 256 << 20
    x = torch.from_numpy(synth.mixed_bytes(n, segment=16 << 20)).cuda()
    ctx = bz.Context(9, 10)
    cap = bz.compress_bound(n)
    z = torch.empty(cap, dtype=torch.uint8, device="cuda")
    zn = ctx.compress_device(x.data_ptr(), n, z.data_ptr(), cap)
    y = torch.empty(n, dtype=torch.uint8, device="cuda")
    with bz.Decompressor(10000) as d:
        got = d.decompress_device(z.data_ptr(), zn, y.data_ptr(), n)
    assert got == n
    assert torch.equal(x, y)


# ---- streaming decode with bounded memory (bz2mi_dstream; the reference's
# block-at-a-time InputStream, InputStream.hpp:51-72,125-158)

def _reader(z: bytes):
    pos = [0]

    def read(k):
        piece = z[pos[0]: pos[0] + k]
        pos[0] += len(piece)
        return piece
    return read


@pytest.mark.parametrize("level", [9, 1])
def test_stream_decode_small_windows(bz, dec, level):
    """Windows far smaller than the stream (blocks cut by window ends, blocks
    that need a longer window, output buffers that hold a few blocks and
    grow when one block needs more) give the whole-input bytes."""
    from bz2mi import synth
    for name, data in [("mixed", synth.mixed_bytes(5 << 20, segment=300 << 10).tobytes()),
                       ("runs_long", synth.runs_bytes(2 << 20, max_run=5000).tobytes()),
                       ("one", b"x"), ("empty", b"")]:
        z = bz.compress(data, level, 10)
        for chunk, window, cap in [(37_000, 150_000, 300_000), (5_000, 20_000, 50_000), (1 << 20, 4 << 20, 8 << 20)]:
            got = b"".join(dec.stream(_reader(z), chunk=chunk, window=window, out_cap=cap))
            assert got == data, (name, level, chunk, window, cap)


def test_stream_decode_golden_and_concatenated(bz, manifest):
    with bz.Decompressor(10000) as d:
        for name, e in sorted(manifest["cases"].items()):
            data = golden_input(name)
            for st in e["streams"]:
                z = golden_file(st["file"])
                assert b"".join(d.stream(_reader(z), chunk=4096, window=16384, out_cap=1 << 16)) == data, name
    a, b = b"first stream " * 5000, b"second" * 7000
    z = bz2.compress(a, 9) + bz2.compress(b, 9) + b"trailing junk"
    with bz.Decompressor(100000, concatenated=True) as d:
        assert b"".join(d.stream(_reader(z), chunk=3000, window=9000, out_cap=1 << 16)) == a + b
    with bz.Decompressor(100000) as d:  # the reference: the first stream only
        assert b"".join(d.stream(_reader(z), chunk=3000, window=9000, out_cap=1 << 16)) == a


def test_stream_decode_error_after_the_good_blocks(bz, dec):
    """A corrupted block in the middle: the blocks before it come out, then the
    reference's message (the same the whole-input call reports)."""
    from bz2mi import synth
    data = synth.random_bytes(3 << 20).tobytes()   # ~35 blocks of 90,000 bytes
    z = bytearray(bz.compress(data, 9, 10))
    z[len(z) // 2] ^= 0x10
    z = bytes(z)
    with pytest.raises(bz.DecompressError) as whole:
        dec.decompress(z)
    got = []
    with pytest.raises(bz.DecompressError) as streamed:
        for piece in dec.stream(_reader(z), chunk=100_000, window=400_000, out_cap=1 << 20):
            got.append(piece)
    got = b"".join(got)
    assert str(streamed.value) == str(whole.value)
    assert len(got) > (1 << 20) and data.startswith(got)


def test_crafted_magics_allocate_bounded_memory(bz):
    """16 MiB of block magics after a stream header: the decoder reports the
    reference's error, and its device memory stays within a few times the
    input (the input's device copy, the candidate list, the table budget)
    instead of growing with the number of matches (~2.8 M here)."""
    import torch
    n = 16 << 20
    z = b"BZh9" + b"1AY&SY" * (n // 6)
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    with bz.Decompressor(10000) as d:
        with pytest.raises(bz.DecompressError):
            d.decompress(z, cap=1 << 20)
        free1, _ = torch.cuda.mem_get_info()
        with pytest.raises(bz.DecompressError):
            for _ in d.stream(_reader(z), chunk=4 << 20, window=8 << 20, out_cap=1 << 20):
                pass
        free2, _ = torch.cuda.mem_get_info()
    used = free0 - min(free1, free2)
    assert used <= 4 * len(z) + (32 << 20), used


def test_device_decode_unaligned_buffers(bz):
    """Input and output device pointers at odd offsets: the input is staged
    (the readers load 4-byte words), the RLE1 pass stores 16-byte blocks by
    address (chunk edges byte-wise) -- the bytes around the output stay."""
    import torch
    from bz2mi import synth
    data = synth.mixed_bytes(3 << 20, segment=256 << 10).tobytes()
    z = bz.compress(data, 9, 10)
    zin = torch.zeros(len(z) + 3, dtype=torch.uint8, device="cuda")
    zin[3:] = torch.frombuffer(bytearray(z), dtype=torch.uint8).cuda()
    y = torch.full((len(data) + 16,), 0xA5, dtype=torch.uint8, device="cuda")
    with bz.Decompressor(10000) as d:
        got = d.decompress_device(zin.data_ptr() + 3, len(z), y.data_ptr() + 5, len(data))
    assert got == len(data)
    out = y.cpu().numpy().tobytes()
    assert out[5:5 + len(data)] == data
    assert out[:5] == b"\xa5" * 5 and out[5 + len(data):] == b"\xa5" * 11


def test_skewed_alphabet_long_codes(bz):
    """A heavily skewed byte distribution: code lengths up to the limit
    (codes longer than the 9-bit lookup take the windowed decoder's
    per-symbol path) and large jumps between consecutive lengths (delta codes
    of more than 15 pairs: the word parser's bit-by-bit fallback)."""
    rng = np.random.default_rng(7)
    p = 0.5 ** np.arange(1, 41)
    p = p / p.sum()
    sym = rng.choice(40, size=3 << 20, p=p).astype(np.uint8)
    data = (sym * 5 + 3).astype(np.uint8).tobytes()
    z = bz.compress(data, 9, 10)
    with bz.Decompressor(10000) as d:
        assert d.decompress(z) == data
    with bz.Decompressor(100000) as d:
        assert d.decompress(bz2.compress(data, 9)) == data
