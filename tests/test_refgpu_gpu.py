"""The HIP path pinned directly to the reference's own MI355X output.

tests/golden/refgpu/ holds streams the unmodified reference (app.cpp +
kernel.cpp through the ROCm OpenCL runtime) wrote on an MI355X
(test_refgpu.py).  Here, on the device:

* bz2mi compresses the same input at the same level / p, and every block's
  split (its CRC over the RLE1 bytes), randomised bit, origPtr (the BWT,
  kernel.cpp:3099-3122), symbol map (:2483-2511) and MTF/RLE2 symbol sequence
  (:2561-2649) are the reference's, as is the stream CRC
  (OutputStream.hpp:163-176, 202).  The Huffman tables differ by hazard H3
  (the reference's uninitialised tableFrequencies, kernel.cpp:2902; O_ref --
  zero per pass -- is the device path's byte-level contract, test_pins.py);
* the HIP decoder reads every reference stream back to the input (the decoder
  analogue of BlockDecompressor.hpp:134-282).
"""
from __future__ import annotations

import hashlib
import os

import pytest

from conftest import GOLDEN, have_gpu
from bz2parse import parse_stream
from test_refgpu import REFGPU, _ids, _input

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not have_gpu(), reason="needs a HIP device")]


@pytest.mark.parametrize("e", REFGPU["streams"], ids=_ids)
def test_device_stream_equals_reference_gpu_upstream_stages(e):
    import bz2mi
    z = open(os.path.join(GOLDEN, e["file"]), "rb").read()
    assert hashlib.sha256(z).hexdigest() == e["sha256"]
    data = _input(e["input"])
    ref = parse_stream(z)
    ours = parse_stream(bz2mi.compress(data, e["level"], e["p"]))
    assert ours["level"] == ref["level"]
    assert ours["stream_crc"] == ref["stream_crc"]
    assert len(ours["blocks"]) == len(ref["blocks"])
    for i, (a, b) in enumerate(zip(ref["blocks"], ours["blocks"])):
        for k in ("crc", "rand", "orig", "present", "symbols"):
            assert a[k] == b[k], (e["file"], i, k)


def test_device_decoder_reads_reference_gpu_streams():
    import bz2mi
    with bz2mi.Decompressor(10000) as d:
        for e in REFGPU["streams"]:
            z = open(os.path.join(GOLDEN, e["file"]), "rb").read()
            assert d.decompress(z) == _input(e["input"]), e["file"]
