"""The reference's CLI, app.cpp, unmodified, compressing on the GPU through the
mirror OutputStream (config C1 literally: "Compress a 10 KB text file at -1
via app.cpp").  The binary is built in the build container by
__graft_entry__.build() (build_reference_app: app.cpp compiled against
bzip2-opencl_amd/include + libbz2mi); its output must be the reference's
bytes: the O_ref fixture for C1, the O_ref hash pins for multi-MiB inputs
handed to the device in several stream units (BZ2MI_UNIT_BYTES)."""
from __future__ import annotations

import hashlib
import os
import subprocess

import pytest

from conftest import PKG, CpuRef, golden_file, golden_input, have_gpu
from test_pins import PINS, pin_input

APP = os.path.join(PKG, "build", "app_bz2mi")
# the reference decoder's messages (std::runtime_error in InputStream.hpp /
# BlockDecompressor.hpp / HuffmanStageDecoder.hpp), which the mirror throws too
REF_DECODE_ERRORS = ("BZip2 block CRC error", "BZip2 stream CRC error", "BZip2 block exceeds declared block size",
                     "BZip2 start pointer invalid", "BZip2 stream format error", "Error decoding  block",
                     "Insufficient data", "Invalid BZip2 header", "block Huffman tables invalid",
                     "BZip2 randomised blocks not implemented")

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not have_gpu(), reason="needs a HIP device"),
              pytest.mark.skipif(not os.path.exists(APP), reason="app.cpp not built (build container step)")]


def _compress(tmp_path, data: bytes, level: int, p: int, unit_bytes: int | None = None) -> bytes:
    src = tmp_path / "in.bin"
    src.write_bytes(data)
    env = dict(os.environ)
    if unit_bytes:
        env["BZ2MI_UNIT_BYTES"] = str(unit_bytes)
    r = subprocess.run([APP, str(src), "-k", "-s", str(level), "-p", str(p)], capture_output=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    out = (tmp_path / "in.bin.bz2").read_bytes()
    (tmp_path / "in.bin.bz2").unlink()
    return out


def test_app_c1_equals_oref(tmp_path):
    got = _compress(tmp_path, golden_input("c1_text10k"), 1, 10)
    assert got == golden_file("oref/c1_text10k.s1.p10.bz2")


@pytest.mark.parametrize("unit_bytes", [None, 1 << 20, 700_001])
@pytest.mark.parametrize("pin", [p for p in PINS["pins"] if p["input"] in ("txt2m75", "mix2m75", "run2m75")
                                 and p["unit"] == 10000 and p["p"] in (10, 3)],
                         ids=lambda p: f"{p['input']}-s{p['level']}-p{p['p']}")
def test_app_matches_oref_pins(tmp_path, pin, unit_bytes):
    got = _compress(tmp_path, pin_input(pin["input"]), pin["level"], pin["p"], unit_bytes)
    assert (len(got), hashlib.sha256(got).hexdigest()) == (pin["bytes"], pin["sha256"])


def test_app_small_and_empty(tmp_path):
    for data in (b"", b"a", b"aa", bytes(range(256)) * 3):
        assert _compress(tmp_path, data, 9, 10, 100_000) == CpuRef().compress(data, 9, 10)


def test_app_checks_fixtures_on_the_device(tmp_path, manifest):
    """app.cpp -c / -d through the mirror InputStream, which decodes on the
    device (bz2mi_decompress): every committed O_ref stream."""
    for name, e in sorted(manifest["cases"].items()):
        for st in e["streams"]:
            p = tmp_path / (name + ".bin.bz2")
            p.write_bytes(golden_file(st["file"]))
            r = subprocess.run([APP, str(p), "-c"], capture_output=True, text=True, timeout=120)
            assert r.returncode == 0 and "Integrity check passed" in r.stdout, (st["file"], r.stderr)
            r = subprocess.run([APP, str(p), "-d", "-k"], capture_output=True, timeout=120)
            assert r.returncode == 0, r.stderr
            out = tmp_path / (name + ".bin")
            assert out.read_bytes() == golden_input(name), st["file"]
            out.unlink()
    bad = bytearray(golden_file("oref/text64k.s9.p10.bz2"))
    bad[len(bad) // 2] ^= 0x10
    p = tmp_path / "bad.bin.bz2"
    p.write_bytes(bytes(bad))
    r = subprocess.run([APP, str(p), "-c"], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "Integrity check passed" not in r.stdout
    assert any(m in r.stderr for m in REF_DECODE_ERRORS), r.stderr


def test_app_round_trip_with_its_decoder(tmp_path):
    data = pin_input("mix2m75")
    z = _compress(tmp_path, data, 9, 10, 1 << 20)
    p = tmp_path / "x.bin.bz2"
    p.write_bytes(z)
    r = subprocess.run([APP, str(p), "-d", "-k"], capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "x.bin").read_bytes() == data
    r = subprocess.run([APP, str(p), "-c"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "Integrity check passed" in r.stdout


def test_app_decodes_in_small_windows(tmp_path):
    """The mirror InputStream decodes in bounded windows (bz2mi_dstream): with
    windows of 200 KB a multi-block file decodes to the same bytes, and a
    corrupted one fails with the reference's message."""
    from bz2mi import synth
    data = synth.mixed_bytes(3 << 20, segment=256 << 10).tobytes()
    src = tmp_path / "w.bin"
    src.write_bytes(data)
    r = subprocess.run([APP, str(src), "-k", "-s", "9", "-p", "10"], capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr
    z = tmp_path / "w.bin.bz2"
    src.unlink()
    env = dict(os.environ, BZ2MI_DSTREAM_WINDOW="200000")
    r = subprocess.run([APP, str(z), "-d", "-k"], capture_output=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr
    assert src.read_bytes() == data
    r = subprocess.run([APP, str(z), "-c"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "Integrity check passed" in r.stdout, (r.stdout, r.stderr)
    bad = bytearray(z.read_bytes())
    bad[len(bad) // 2] ^= 0x08
    zb = tmp_path / "bad.bin.bz2"
    zb.write_bytes(bytes(bad))
    r = subprocess.run([APP, str(zb), "-c"], capture_output=True, text=True, env=env, timeout=300)
    # app.cpp catches nothing: the decoder's exception ends the process with the
    # reference's message (include/InputStream.hpp / BlockDecompressor.hpp)
    assert r.returncode != 0 and "Integrity check passed" not in r.stdout, (r.stdout, r.stderr)
    assert any(m in r.stderr for m in REF_DECODE_ERRORS), r.stderr
