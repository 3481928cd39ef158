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
