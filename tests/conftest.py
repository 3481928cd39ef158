"""Shared test helpers.  Markers: `gpu` (needs an MI355X; run with -m gpu)."""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "bzip2-opencl_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
REF = os.environ.get("BZ2MI_REFERENCE", "/root/reference")
sys.path.insert(0, PKG)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")


def _make(target_dir, *targets):
    subprocess.run(["make", "-C", target_dir, *targets], check=True, stdout=subprocess.DEVNULL,
                   stderr=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_input(name: str) -> bytes:
    with open(os.path.join(GOLDEN, "inputs", name + ".bin"), "rb") as f:
        return f.read()


def golden_file(rel: str) -> bytes:
    with open(os.path.join(GOLDEN, rel), "rb") as f:
        return f.read()


class CpuRef:
    """ctypes view of the C restatement (oracle/_build/libcpuref.so)."""

    def __init__(self):
        path = os.path.join(REPO, "oracle", "_build", "libcpuref.so")
        if not os.path.exists(path):
            _make(os.path.join(REPO, "oracle"), "cpu")
        L = ctypes.CDLL(path)
        c = ctypes
        L.cpuref_compress.restype = c.c_longlong
        L.cpuref_compress.argtypes = [c.c_char_p, c.c_size_t, c.c_int, c.c_int, c.c_int, c.c_char_p, c.c_size_t,
                                      c.c_int]
        L.cpuref_bound.restype = c.c_size_t
        L.cpuref_bound.argtypes = [c.c_size_t, c.c_int, c.c_int]
        L.cpuref_bwt.restype = c.c_int
        L.cpuref_bwt.argtypes = [c.c_char_p, c.c_int, c.c_char_p]
        L.cpuref_mtf.restype = c.c_int
        L.cpuref_mtf.argtypes = [c.c_char_p, c.c_int, c.c_char_p, c.c_void_p, c.c_void_p, c.POINTER(c.c_int)]
        L.cpuref_split.restype = c.c_longlong
        L.cpuref_split.argtypes = [c.c_char_p, c.c_size_t, c.c_int, c.c_char_p, c.c_size_t, c.c_void_p,
                                   c.c_void_p, c.c_void_p, c.c_size_t]
        L.cpuref_block_payload.restype = c.c_longlong
        L.cpuref_block_payload.argtypes = [c.c_int, c.c_char_p, c.c_void_p, c.c_int, c.c_int, c.c_void_p,
                                           c.c_char_p, c.c_uint64, c.c_void_p, c.c_void_p]
        self.L = L

    def compress(self, data: bytes, level=9, p=10, unit=10000, threads=4) -> bytes:
        cap = self.L.cpuref_bound(len(data), level, unit)
        out = ctypes.create_string_buffer(cap)
        n = self.L.cpuref_compress(data, len(data), level, p, unit, out, cap, threads)
        assert n >= 0, n
        return out.raw[:n]

    def bwt(self, block: bytes):
        out = ctypes.create_string_buffer(max(1, len(block)))
        orig = self.L.cpuref_bwt(block, len(block), out)
        return out.raw[: len(block)], orig

    def mtf(self, bwt: bytes, present: bytes):
        import numpy as np
        sym = np.zeros(len(bwt) + 2, dtype=np.uint16)
        hist = np.zeros(258, dtype=np.uint32)
        alpha = ctypes.c_int(0)
        m = self.L.cpuref_mtf(bwt, len(bwt), present, sym.ctypes.data, hist.ctypes.data, ctypes.byref(alpha))
        return sym[:m], hist, alpha.value

    def split(self, data: bytes, S: int):
        nb = self.L.cpuref_split(data, len(data), S, None, 0, None, None, None, 0)
        nb = -nb if nb < 0 else nb
        stride = S + 8
        blocks = ctypes.create_string_buffer(max(1, nb * stride))
        lens = (ctypes.c_uint32 * max(1, nb))()
        crcs = (ctypes.c_uint32 * max(1, nb))()
        self.L.cpuref_split(data, len(data), S, blocks, stride, None, lens, crcs, nb)
        return [blocks.raw[b * stride: b * stride + lens[b]] for b in range(nb)], list(crcs)[:nb]


@pytest.fixture(scope="session")
def cpuref():
    return CpuRef()


class CpuRefUnit:
    """The unit protocol (include/bz2mi.h bz2mi_unit_*) on the C restatement
    (cpuref_unit_*), for driving bz2mi.shard on CPU ranks."""

    def __init__(self, level=9, parallel=10, unit=10000, threads=2):
        self.L = CpuRef().L
        c = ctypes
        L = self.L
        L.cpuref_unit_open.restype = c.c_void_p
        L.cpuref_unit_open.argtypes = [c.c_char_p, c.c_size_t, c.c_size_t, c.c_int, c.c_int, c.c_int, c.c_int,
                                       c.c_uint64, c.c_uint64, c.POINTER(c.c_uint64), c.POINTER(c.c_uint64), c.c_int]
        L.cpuref_unit_sums.argtypes = [c.c_void_p, c.c_void_p]
        L.cpuref_unit_encode.restype = c.c_int
        L.cpuref_unit_encode.argtypes = [c.c_void_p, c.c_void_p, c.POINTER(c.c_uint64), c.POINTER(c.c_uint32),
                                         c.c_int]
        L.cpuref_unit_assemble.restype = c.c_longlong
        L.cpuref_unit_assemble.argtypes = [c.c_void_p, c.c_uint64, c.c_uint32, c.c_int, c.c_char_p, c.c_size_t]
        L.cpuref_unit_free.argtypes = [c.c_void_p]
        self.level, self.parallel, self.unit, self.threads = level, parallel, unit, threads
        self.h = None

    def begin(self, buf: bytes, n_own: int, n_halo: int, ends: bool):
        self.buf = bytes(buf)
        self.n_own, self.n_halo, self.ends = n_own, n_halo, ends

    def chain(self, entry, first_block):
        ex = ctypes.c_uint64(0)
        nb = ctypes.c_uint64(0)
        self.h = self.L.cpuref_unit_open(self.buf, self.n_own, self.n_halo, 1 if self.ends else 0, self.level,
                                         self.parallel, self.unit, entry, first_block, ctypes.byref(ex),
                                         ctypes.byref(nb), self.threads)
        assert self.h, "cpuref_unit_open failed (halo too short?)"
        return ex.value, nb.value

    def sums(self):
        import numpy as np
        out = np.zeros(self.parallel * 258, dtype=np.uint32)
        self.L.cpuref_unit_sums(self.h, out.ctypes.data)
        return out

    def encode(self, carried):
        import numpy as np
        c = np.ascontiguousarray(carried, dtype=np.uint32)
        bits = ctypes.c_uint64(0)
        crc = ctypes.c_uint32(0)
        assert self.L.cpuref_unit_encode(self.h, c.ctypes.data, ctypes.byref(bits), ctypes.byref(crc),
                                         self.threads) == 0
        self.bits = bits.value
        return bits.value, crc.value

    def assemble(self, bit_offset, crc_before, flags):
        cap = (self.bits + 32 + 80) // 8 + 16
        out = ctypes.create_string_buffer(cap)
        n = self.L.cpuref_unit_assemble(self.h, bit_offset, crc_before, flags, out, cap)
        assert n >= 0
        return out.raw[:n]

    def __del__(self):
        if getattr(self, "h", None):
            self.L.cpuref_unit_free(self.h)
            self.h = None


def unit_buffers(data: bytes, cuts: list[int], halo: int):
    """Split a stream at `cuts` into unit buffers: (bytes own+halo, n_own, n_halo, ends)."""
    bounds = [0] + list(cuts) + [len(data)]
    out = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        end = min(len(data), b + halo)
        out.append((data[a:end], b - a, end - b, end == len(data)))
    return out


def oref_lib():
    path = os.path.join(REPO, "oracle", "_ref", "liboref.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.oref_compress.restype = ctypes.c_longlong
    L.oref_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_char_p, ctypes.c_size_t]
    return L


def have_gpu() -> bool:
    try:
        import bz2mi
        return bz2mi.lib().bz2mi_device_count() > 0
    except Exception:
        return False
