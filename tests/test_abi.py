"""The drop-in boundary, checked without a GPU.

* libbz2mi.so loads and exports every function include/bz2mi.h declares;
* without a HIP device the library fails loudly (NULL context + message),
  it never falls back to a CPU path;
* the C++ mirror headers compile; their host decoder (InputStream) reads every
  golden stream; BlockCompressor reproduces the reference's RLE1 block split;
* the reference's own app.cpp compiles unchanged against the mirror headers
  and links against libbz2mi.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess

import pytest

from conftest import PKG, REF, REPO, golden_file, golden_input, have_gpu

HEADER = os.path.join(REPO, "include", "bz2mi.h")
LIB = os.path.join(PKG, "bz2mi", "libbz2mi.so")


def _ensure_lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, stdout=subprocess.DEVNULL)


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bz2mi_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    _ensure_lib()
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (bz2mi_\w+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    import bz2mi
    assert set(declared_functions()) == set(bz2mi.EXPORTS)


def test_python_binding_resolves_symbols():
    _ensure_lib()
    import bz2mi
    L = bz2mi.lib()
    for name in bz2mi.EXPORTS:
        assert getattr(L, name) is not None
    assert bz2mi.compress_bound(10 ** 6, 9, 10000) > 10 ** 6


@pytest.mark.skipif(have_gpu(), reason="checks the no-device failure path")
def test_no_device_fails_loudly():
    _ensure_lib()
    import bz2mi
    with pytest.raises(RuntimeError):
        bz2mi.Context(9, 10)
    with pytest.raises(ValueError):
        bz2mi.OutputStream(open(os.devnull, "wb"), 10, 10)
    with pytest.raises(ValueError):
        bz2mi.OutputStream(open(os.devnull, "wb"), 9, 0)


HARNESS = r"""
#include <fstream>
#include <iostream>
#include <sstream>
#include <vector>
#include "InputStream.hpp"
#include "BlockCompressor.hpp"
int main(int argc, char** argv) {
    std::string mode = argv[1];
    std::ifstream f(argv[2], std::ios::binary);
    std::stringstream ss; ss << f.rdbuf();
    std::string in = ss.str();
    if (mode == "decode") {
        std::istringstream is(in);
        InputStream s(is);
        std::string out; int c;
        while ((c = s.read()) != -1) out.push_back((char)c);
        s.close();
        std::cout.write(out.data(), out.size());
        return 0;
    }
    // split: block lengths and CRCs of the RLE1 front end at block size argv[3]
    int S = std::atoi(argv[3]);
    std::vector<unsigned char> blk(S + 8);
    std::vector<bool> dummy;
    bool present[256];
    BlockCompressor bc(blk.data(), present, S);
    bc.reset();
    for (size_t i = 0; i < in.size(); ++i) {
        if (!bc.write((unsigned char)in[i])) {
            bc.finishRLE();
            std::cout << bc.getBlockLength() << " " << (unsigned)bc.getCRC() << "\n";
            bc.reset();
            bc.write((unsigned char)in[i]);
        }
    }
    if (!bc.isEmpty()) { bc.finishRLE(); std::cout << bc.getBlockLength() << " " << (unsigned)bc.getCRC() << "\n"; }
    return 0;
}
"""


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("hdr")
    src = d / "h.cpp"
    src.write_text(HARNESS)
    exe = d / "h"
    _ensure_lib()
    lib = os.path.dirname(LIB)
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(PKG, "include"),
                    "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe), "-L", lib, "-lbz2mi",
                    "-Wl,-rpath," + lib], check=True)
    return str(exe)


# the CPU tests run the mirror InputStream's host decoder (the device decoder
# is its default; tests/test_app_gpu.py covers that path)
HOST_DEC = dict(os.environ, BZ2MI_HOST_DECODER="1")


def test_mirror_decoder_reads_golden_streams(harness, manifest, tmp_path):
    for name, e in sorted(manifest["cases"].items()):
        data = golden_input(name)
        for st in e["streams"]:
            p = tmp_path / "x.bz2"
            p.write_bytes(golden_file(st["file"]))
            out = subprocess.run([harness, "decode", str(p)], capture_output=True, check=True, env=HOST_DEC).stdout
            assert out == data, (name, st)


def test_mirror_decoder_rejects_corruption(harness, tmp_path):
    good = bytearray(golden_file("oref/text64k.s9.p10.bz2"))
    good[len(good) // 2] ^= 0x10
    p = tmp_path / "bad.bz2"
    p.write_bytes(bytes(good))
    r = subprocess.run([harness, "decode", str(p)], capture_output=True, env=HOST_DEC)
    assert r.returncode != 0  # std::runtime_error (CRC / table / format)


def test_mirror_blockcompressor_split(harness, cpuref, tmp_path):
    for name in ("runs64k", "h1_exact", "text64k", "fb_const"):
        data = golden_input(name)
        p = tmp_path / "in.bin"
        p.write_bytes(data)
        for S in (10000, 90000):
            out = subprocess.run([harness, "split", str(p), str(S)], capture_output=True, check=True, text=True).stdout
            got = [tuple(map(int, l.split())) for l in out.splitlines()]
            blocks, crcs = cpuref.split(data, S)
            assert got == [(len(b), c) for b, c in zip(blocks, crcs)], (name, S)


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "app.cpp")), reason="reference app.cpp not present")
def test_reference_app_compiles_unchanged(tmp_path, manifest):
    """The reference CLI, byte-for-byte, against the mirror headers + libbz2mi."""
    _ensure_lib()
    shutil.copy(os.path.join(REF, "app.cpp"), tmp_path / "app.cpp")  # build-time copy only
    os.symlink(os.path.join(PKG, "include"), tmp_path / "include")
    exe = tmp_path / "app"
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(REPO, "include"), str(tmp_path / "app.cpp"),
                    "-o", str(exe), "-L", os.path.dirname(LIB), "-lbz2mi",
                    "-Wl,-rpath," + os.path.dirname(LIB)], check=True)
    # its decoder path runs on the host: -d and -c on golden streams
    data = golden_input("c1_text10k")
    src = tmp_path / "c1.bin.bz2"
    src.write_bytes(golden_file("oref/c1_text10k.s1.p10.bz2"))
    r = subprocess.run([str(exe), str(src), "-d", "-k"], capture_output=True, cwd=tmp_path, env=HOST_DEC)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "c1.bin").read_bytes() == data
    r = subprocess.run([str(exe), str(src), "-c"], capture_output=True, text=True, cwd=tmp_path, env=HOST_DEC)
    assert r.returncode == 0 and "Integrity check passed" in r.stdout
