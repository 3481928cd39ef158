"""bz2mi -- Python binding of libbz2mi (MI355X-native bzip2 block compression).

Thin ctypes layer over the C ABI declared in include/bz2mi.h.  The shared
library is built in-tree (``make -C bzip2-opencl_amd``) and always loaded from
this directory; there is no CPU fallback -- importing works without a GPU, but
every compression call needs the HIP device and fails loudly otherwise.

Reference interface mirrored: OutputStream(std::ostream&, level, parallel)
/ write / close (Stan1slav337/Bzip2-OpenCL include/OutputStream.hpp:65-176),
with the same argument meaning and the same errors (ValueError for
std::invalid_argument, RuntimeError for std::runtime_error).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# BZ2MI_LIBRARY: an alternative build of the library (A/B experiments)
LIB_PATH = os.environ.get("BZ2MI_LIBRARY") or os.path.join(_HERE, "libbz2mi.so")

BZ2MI_OK = 0
ABI_VERSION = 5  # include/bz2mi.h BZ2MI_ABI_VERSION
BZ2MI_EINVAL = -1
BZ2MI_EDEVICE = -2
BZ2MI_ESPACE = -3
BZ2MI_ESTATE = -4
BZ2MI_EFORMAT = -5

# every symbol include/bz2mi.h declares
EXPORTS = (
    "bz2mi_last_error", "bz2mi_device_count", "bz2mi_version", "bz2mi_create", "bz2mi_destroy",
    "bz2mi_compress_bound", "bz2mi_compress_rle1", "bz2mi_finish", "bz2mi_compress_blocks",
    "bz2mi_compress", "bz2mi_compress_device", "bz2mi_last_timings", "bz2mi_blocks_done",
    "bz2mi_last_stats", "bz2mi_dcreate", "bz2mi_ddestroy", "bz2mi_dset_flags", "bz2mi_decompress", "bz2mi_decompress_device",
    "bz2mi_dlast_timings", "bz2mi_unit_halo", "bz2mi_unit_create", "bz2mi_unit_destroy", "bz2mi_unit_begin",
    "bz2mi_unit_chain", "bz2mi_unit_speculate", "bz2mi_unit_chain_info", "bz2mi_unit_sums", "bz2mi_unit_encode",
    "bz2mi_unit_assemble", "bz2mi_unit_timings",
    "bz2mi_unit_stats", "bz2mi_host_alloc", "bz2mi_host_free", "bz2mi_unit_begin_host", "bz2mi_unit_assemble_host",
    "bz2mi_dstream_reset", "bz2mi_dstream", "bz2mi_dlast_trailing", "bz2mi_abi_version",
)

_lib = None


def lib() -> ctypes.CDLL:
    """Load libbz2mi.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libbz2mi.so not built: run `make -C {os.path.dirname(_HERE)}` ({LIB_PATH})")
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7.  If
    # torch is importable it is loaded first, so libbz2mi's libamdhip64.so.7
    # dependency binds to that same runtime (same SONAME) and device pointers,
    # streams and devices are shared; otherwise the system ROCm runtime is used.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    c = ctypes
    L.bz2mi_last_error.restype = c.c_char_p
    L.bz2mi_device_count.restype = c.c_int
    L.bz2mi_version.restype = c.c_char_p
    L.bz2mi_create.restype = c.c_void_p
    L.bz2mi_create.argtypes = [c.c_int, c.c_int, c.c_int, c.c_int]
    L.bz2mi_destroy.argtypes = [c.c_void_p]
    L.bz2mi_compress_bound.restype = c.c_size_t
    L.bz2mi_compress_bound.argtypes = [c.c_size_t, c.c_int, c.c_int]
    L.bz2mi_compress_rle1.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_void_p, c.c_uint32,
                                      c.c_void_p, c.c_size_t, c.POINTER(c.c_size_t)]
    L.bz2mi_finish.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.POINTER(c.c_size_t)]
    L.bz2mi_compress_blocks.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_uint32, c.c_void_p,
                                        c.c_size_t, c.c_void_p]
    L.bz2mi_compress.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t,
                                 c.POINTER(c.c_size_t)]
    L.bz2mi_compress_device.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t,
                                        c.POINTER(c.c_size_t), c.c_void_p]
    L.bz2mi_last_timings.argtypes = [c.c_void_p, c.POINTER(c.c_float)]
    L.bz2mi_last_stats.restype = c.c_int
    L.bz2mi_last_stats.argtypes = [c.c_void_p, c.POINTER(c.c_uint64)]
    L.bz2mi_blocks_done.restype = c.c_uint64
    L.bz2mi_blocks_done.argtypes = [c.c_void_p]
    L.bz2mi_dcreate.restype = c.c_void_p
    L.bz2mi_dcreate.argtypes = [c.c_int, c.c_int]
    L.bz2mi_ddestroy.argtypes = [c.c_void_p]
    L.bz2mi_dset_flags.restype = c.c_int
    L.bz2mi_dset_flags.argtypes = [c.c_void_p, c.c_int]
    L.bz2mi_decompress.restype = c.c_int
    L.bz2mi_decompress.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t,
                                   c.POINTER(c.c_size_t)]
    L.bz2mi_decompress_device.restype = c.c_int
    L.bz2mi_decompress_device.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t,
                                          c.POINTER(c.c_size_t), c.c_void_p]
    if hasattr(L, "bz2mi_dstream"):  # (older A/B builds lack it; test_abi checks the product library)
        L.bz2mi_dstream_reset.restype = c.c_int
        L.bz2mi_dstream_reset.argtypes = [c.c_void_p]
        L.bz2mi_dstream.restype = c.c_int
        L.bz2mi_dstream.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_uint, c.c_int, c.c_void_p,
                                    c.c_size_t, c.POINTER(c.c_uint64), c.POINTER(c.c_size_t), c.POINTER(c.c_int)]
    L.bz2mi_dlast_timings.restype = c.c_int
    L.bz2mi_dlast_timings.argtypes = [c.c_void_p, c.POINTER(c.c_float)]
    if hasattr(L, "bz2mi_abi_version"):
        L.bz2mi_dlast_trailing.restype = c.c_int
        L.bz2mi_dlast_trailing.argtypes = [c.c_void_p, c.POINTER(c.c_uint64)]
        L.bz2mi_abi_version.restype = c.c_int
        if L.bz2mi_abi_version() != ABI_VERSION:
            raise RuntimeError(f"{LIB_PATH}: ABI {L.bz2mi_abi_version()}, this binding expects {ABI_VERSION}")
    elif not os.environ.get("BZ2MI_LIBRARY"):  # (an older library loaded on purpose for an A/B run)
        raise RuntimeError(f"{LIB_PATH}: no bz2mi_abi_version (a library older than ABI {ABI_VERSION})")
    L.bz2mi_unit_halo.restype = c.c_size_t
    L.bz2mi_unit_halo.argtypes = [c.c_int, c.c_int]
    L.bz2mi_unit_create.restype = c.c_void_p
    L.bz2mi_unit_create.argtypes = [c.c_void_p]
    L.bz2mi_unit_destroy.argtypes = [c.c_void_p]
    L.bz2mi_unit_begin.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_size_t, c.c_int, c.c_void_p]
    L.bz2mi_unit_chain.argtypes = [c.c_void_p, c.c_uint64, c.c_uint64, c.POINTER(c.c_uint64), c.POINTER(c.c_uint64)]
    L.bz2mi_unit_speculate.argtypes = [c.c_void_p, c.POINTER(c.c_uint64)]
    L.bz2mi_unit_chain_info.argtypes = [c.c_void_p, c.POINTER(c.c_uint64)]
    L.bz2mi_unit_sums.argtypes = [c.c_void_p, c.c_void_p]
    L.bz2mi_unit_encode.argtypes = [c.c_void_p, c.c_void_p, c.POINTER(c.c_uint64), c.POINTER(c.c_uint32)]
    L.bz2mi_unit_assemble.argtypes = [c.c_void_p, c.c_uint64, c.c_uint32, c.c_int, c.c_void_p, c.c_size_t,
                                      c.POINTER(c.c_size_t), c.c_void_p]
    L.bz2mi_unit_timings.argtypes = [c.c_void_p, c.POINTER(c.c_float)]
    L.bz2mi_unit_stats.argtypes = [c.c_void_p, c.POINTER(c.c_uint64)]
    for name in ("bz2mi_unit_begin", "bz2mi_unit_chain", "bz2mi_unit_speculate", "bz2mi_unit_chain_info",
                 "bz2mi_unit_sums", "bz2mi_unit_encode",
                 "bz2mi_unit_assemble", "bz2mi_unit_timings", "bz2mi_unit_stats"):
        getattr(L, name).restype = c.c_int
    # debugging entry points (not in include/bz2mi.h)
    L.bz2mi_debug_selftest.restype = c.c_int
    L.bz2mi_debug_selftest.argtypes = [c.POINTER(c.c_uint32), c.c_int]
    L.bz2mi_debug_phases.restype = c.c_int
    L.bz2mi_debug_phases.argtypes = [c.c_int, c.POINTER(c.c_ulonglong)]
    for name in ("bz2mi_compress_rle1", "bz2mi_finish", "bz2mi_compress_blocks", "bz2mi_compress",
                 "bz2mi_compress_device", "bz2mi_last_timings"):
        getattr(L, name).restype = c.c_int
    _lib = L
    return L


def _check(rc: int) -> None:
    if rc == BZ2MI_OK:
        return
    msg = lib().bz2mi_last_error().decode(errors="replace")
    if rc == BZ2MI_EINVAL:
        raise ValueError(msg)
    raise RuntimeError(msg or f"bz2mi error {rc}")


def compress_bound(n: int, level: int = 9, unit: int = 10000) -> int:
    return int(lib().bz2mi_compress_bound(n, level, unit))


def _ptr(buf) -> int:
    """Address of a bytes-like / numpy buffer (host memory)."""
    import numpy as np
    a = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
    return a.ctypes.data


class Context:
    """A bz2mi_ctx: one compressed stream on one device (level, p, unit)."""

    def __init__(self, level: int = 9, parallel: int = 10, unit: int = 10000, device: int = 0):
        L = lib()
        h = L.bz2mi_create(level, parallel, unit, device)
        if not h:
            msg = L.bz2mi_last_error().decode(errors="replace")
            if "Invalid" in msg:
                raise ValueError(msg)
            raise RuntimeError(msg)
        self._h = h
        self.level, self.parallel, self.unit = level, parallel, unit
        self.block_size = level * unit
        import weakref
        self._units = weakref.WeakSet()  # units on this context: closed before it

    def close(self) -> None:
        if getattr(self, "_h", None):
            for u in list(self._units):
                u.close()
            lib().bz2mi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self) -> int:
        return self._h

    def compress(self, data) -> bytes:
        """Whole stream: host RLE1 front end + device path + framing."""
        import numpy as np
        src = np.frombuffer(bytes(data) if not isinstance(data, (bytes, bytearray, np.ndarray)) else data,
                            dtype=np.uint8)
        cap = compress_bound(src.size, self.level, self.unit)
        out = np.empty(cap, dtype=np.uint8)
        n = ctypes.c_size_t(0)
        _check(lib().bz2mi_compress(self._h, src.ctypes.data if src.size else None, src.size,
                                    out.ctypes.data, cap, ctypes.byref(n)))
        return out[: n.value].tobytes()

    def compress_blocks(self, blocks: list[bytes]):
        """Payload bits of RLE1 blocks (kernel_close analogue): list of (bytes, nbits)."""
        import numpy as np
        nb = len(blocks)
        stride = max(16, max(len(b) for b in blocks))
        buf = np.zeros(nb * stride, dtype=np.uint8)
        for j, b in enumerate(blocks):
            buf[j * stride: j * stride + len(b)] = np.frombuffer(b, dtype=np.uint8)
        lens = np.array([len(b) for b in blocks], dtype=np.uint32)
        ostride = self.block_size * 3 + 65536
        out = np.zeros(nb * ostride, dtype=np.uint8)
        bits = np.zeros(nb, dtype=np.uint64)
        _check(lib().bz2mi_compress_blocks(self._h, buf.ctypes.data, stride, lens.ctypes.data, nb,
                                           out.ctypes.data, ostride, bits.ctypes.data))
        res = []
        for j in range(nb):
            nbytes = (int(bits[j]) + 7) // 8
            res.append((out[j * ostride: j * ostride + nbytes].tobytes(), int(bits[j])))
        return res

    def compress_device(self, d_in_ptr: int, n: int, d_out_ptr: int, cap: int, stream: int = 0) -> int:
        """Device-resident whole stream; returns the compressed size.  `stream`
        is the hipStream_t the input was written on (0: the null stream)."""
        out_len = ctypes.c_size_t(0)
        _check(lib().bz2mi_compress_device(self._h, d_in_ptr, n, d_out_ptr, cap, ctypes.byref(out_len),
                                           ctypes.c_void_p(stream)))
        return out_len.value

    def stats(self):
        """Volumes of the last compress_device call (enables collection)."""
        arr = (ctypes.c_uint64 * 8)()
        _check(lib().bz2mi_last_stats(self._h, arr))
        keys = ("input_bytes", "blocks", "rle1_bytes", "mtf_symbols", "payload_bits", "output_bytes", "batch_blocks")
        return dict(zip(keys, [int(v) for v in list(arr)[:7]]))

    def timings(self):
        arr = (ctypes.c_float * 6)()
        _check(lib().bz2mi_last_timings(self._h, arr))
        return dict(zip(("front", "bwt", "mtf", "seed", "huffman", "assemble"), list(arr)))


def unit_halo(level: int = 9, unit: int = 10000) -> int:
    """Tail-halo bytes a stream unit needs (bz2mi_unit_halo)."""
    return int(lib().bz2mi_unit_halo(level, unit))


class Unit:
    """A bz2mi_unit: one contiguous piece of a logical stream (include/bz2mi.h
    "one logical stream compressed in units"; driven by bz2mi.shard)."""

    def __init__(self, ctx: Context):
        L = lib()
        h = L.bz2mi_unit_create(ctx.handle)
        if not h:
            raise RuntimeError(L.bz2mi_last_error().decode(errors="replace"))
        self._h = h
        self.ctx = ctx  # keeps the context alive
        self.parallel = ctx.parallel
        ctx._units.add(self)

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().bz2mi_unit_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def begin(self, d_ptr: int, n_own: int, n_halo: int, flags: int = 0, stream: int = 0) -> None:
        _check(lib().bz2mi_unit_begin(self._h, d_ptr, n_own, n_halo, flags, ctypes.c_void_p(stream)))

    def speculate(self) -> int:
        """bz2mi_unit_speculate: chain from the unit's first byte while the
        entry is on its way; returns the speculative block count."""
        nb = ctypes.c_uint64(0)
        _check(lib().bz2mi_unit_speculate(self._h, ctypes.byref(nb)))
        return nb.value

    def chain_info(self) -> dict:
        v = (ctypes.c_uint64 * 4)()
        _check(lib().bz2mi_unit_chain_info(self._h, v))
        return {"spec_blocks": v[0], "spliced": v[1], "chained": v[2], "speculated": bool(v[3])}

    def chain(self, entry: int, first_block: int):
        ex = ctypes.c_uint64(0)
        nb = ctypes.c_uint64(0)
        _check(lib().bz2mi_unit_chain(self._h, entry, first_block, ctypes.byref(ex), ctypes.byref(nb)))
        return ex.value, nb.value

    def sums(self):
        import numpy as np
        out = np.zeros(self.parallel * 258, dtype=np.uint32)
        _check(lib().bz2mi_unit_sums(self._h, out.ctypes.data))
        return out

    def encode(self, carried):
        import numpy as np
        c = np.ascontiguousarray(carried, dtype=np.uint32)
        bits = ctypes.c_uint64(0)
        crc = ctypes.c_uint32(0)
        _check(lib().bz2mi_unit_encode(self._h, c.ctypes.data, ctypes.byref(bits), ctypes.byref(crc)))
        return bits.value, crc.value

    def assemble(self, bit_offset: int, crc_before: int, flags: int, d_out_ptr: int, cap: int,
                 stream: int = 0) -> int:
        """`stream`: the hipStream_t whose queued work may still use the
        output buffer (0: the null stream); assembly waits for it."""
        n = ctypes.c_size_t(0)
        _check(lib().bz2mi_unit_assemble(self._h, bit_offset, crc_before, flags, d_out_ptr, cap, ctypes.byref(n),
                                         ctypes.c_void_p(stream)))
        return n.value

    def timings(self):
        arr = (ctypes.c_float * 6)()
        _check(lib().bz2mi_unit_timings(self._h, arr))
        return dict(zip(("front", "chain", "bwt", "mtf", "huffman", "assemble"), list(arr)))

    def stats(self):
        """Volumes once encoded: RLE1 bytes, MTF/RLE2 symbols, payload bits, blocks."""
        arr = (ctypes.c_uint64 * 4)()
        _check(lib().bz2mi_unit_stats(self._h, arr))
        return dict(zip(("rle1_bytes", "mtf_symbols", "payload_bits", "blocks"), [int(v) for v in arr]))


class DecompressError(RuntimeError):
    """Corrupt .bz2 data: the reference's std::runtime_error (its message)."""


DEC_CONCATENATED = 1


class Decompressor:
    """A bz2mi_dctx: device decoder of .bz2 streams (the reference's
    InputStream / BlockDecompressor / HuffmanStageDecoder, InputStream.hpp:36-159).
    `unit` 10000 accepts the reference's block sizes, 100000 stock bzip2 files.
    `concatenated`: decode every stream of the input (bzip2's behaviour); by
    default only the first, as the reference's InputStream does."""

    last_trailing = 0  # input bytes after the last decoded stream (ignored) of the last decompress()

    def __init__(self, unit: int = 10000, device: int = 0, concatenated: bool = False):
        L = lib()
        h = L.bz2mi_dcreate(unit, device)
        if not h:
            msg = L.bz2mi_last_error().decode(errors="replace")
            raise (ValueError if "Invalid" in msg else RuntimeError)(msg)
        self._h = h
        self.unit = unit
        if concatenated:
            _check(L.bz2mi_dset_flags(h, DEC_CONCATENATED))

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().bz2mi_ddestroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @staticmethod
    def _raise(rc: int) -> None:
        msg = lib().bz2mi_last_error().decode(errors="replace")
        if rc == BZ2MI_EFORMAT:
            raise DecompressError(msg)
        _check(rc)

    def decompress(self, data, cap: int | None = None) -> bytes:
        """Host bytes in, host bytes out (the buffer grows once if too small)."""
        import numpy as np
        src = np.frombuffer(bytes(data), dtype=np.uint8)
        cap = cap if cap is not None else max(1 << 16, src.size * 8)
        for _ in range(2):
            out = np.empty(max(cap, 1), dtype=np.uint8)
            n = ctypes.c_size_t(0)
            rc = lib().bz2mi_decompress(self._h, src.ctypes.data if src.size else None, src.size,
                                        out.ctypes.data, cap, ctypes.byref(n))
            if rc == BZ2MI_ESPACE:
                cap = n.value
                continue
            if rc != BZ2MI_OK:
                self._raise(rc)
            tr = ctypes.c_uint64(0)
            _check(lib().bz2mi_dlast_trailing(self._h, ctypes.byref(tr)))
            self.last_trailing = tr.value
            if tr.value and bytes(src[src.size - tr.value:src.size - tr.value + 3]) == b"BZh":
                import warnings
                warnings.warn(f"{tr.value} bytes after the end of the first stream start another .bz2 stream and "
                              "were not decoded (the reference's InputStream reads one stream; "
                              "Decompressor(concatenated=True) decodes them all)", stacklevel=2)
            return out[: n.value].tobytes()
        raise RuntimeError("decompress: output size changed between attempts")

    def decompress_device(self, d_in_ptr: int, n: int, d_out_ptr: int, cap: int, stream: int = 0) -> int:
        """Device buffers; returns the decompressed size (raises on errors;
        on a short buffer RuntimeError names the size needed)."""
        out_len = ctypes.c_size_t(0)
        rc = lib().bz2mi_decompress_device(self._h, d_in_ptr, n, d_out_ptr, cap, ctypes.byref(out_len),
                                           ctypes.c_void_p(stream) if stream else None)
        if rc == BZ2MI_ESPACE:
            raise RuntimeError(f"output buffer too small: {out_len.value} bytes needed")
        if rc != BZ2MI_OK:
            self._raise(rc)
        return out_len.value

    def stream(self, reader, chunk: int = 16 << 20, window: int = 64 << 20, out_cap: int = 64 << 20):
        """Streaming decode with bounded memory (bz2mi_dstream): `reader(k)`
        returns up to k more compressed bytes (b"" at the end); yields the
        decoded bytes window by window.  Host memory stays O(window + out_cap)."""
        import numpy as np
        L = lib()
        _check(L.bz2mi_dstream_reset(self._h))
        win = bytearray()
        bit = 0
        eof = False
        out = np.empty(out_cap, dtype=np.uint8)
        want = window
        while True:
            while not eof and len(win) < want:
                piece = reader(chunk)
                if not piece:
                    eof = True
                else:
                    win += piece
            src = np.frombuffer(bytes(win), dtype=np.uint8)
            end = ctypes.c_uint64(0)
            n = ctypes.c_size_t(0)
            fin = ctypes.c_int(0)
            rc = L.bz2mi_dstream(self._h, src.ctypes.data if src.size else None, src.size, bit, 1 if eof else 0,
                                 out.ctypes.data, out.size, ctypes.byref(end), ctypes.byref(n), ctypes.byref(fin))
            if rc == BZ2MI_ESPACE:
                out = np.empty(n.value + (n.value >> 3) + 4096, dtype=np.uint8)
                continue
            if rc != BZ2MI_OK:
                self._raise(rc)
            del win[: end.value // 8]
            bit = end.value & 7
            if n.value:
                yield out[: n.value].tobytes()
                want = window
            elif fin.value:
                return
            elif eof:
                raise DecompressError("Insufficient data")
            else:
                want = len(win) + window
            if fin.value:
                return

    def timings(self):
        arr = (ctypes.c_float * 6)()
        _check(lib().bz2mi_dlast_timings(self._h, arr))
        return dict(zip(("scan", "huffman", "mtf", "ibwt", "rle1", "total"), list(arr)))


def decompress(data, unit: int = 10000, device: int = 0, concatenated: bool = False) -> bytes:
    """Whole .bz2 -> bytes, decoded on the device (the first stream, or every
    stream with `concatenated`)."""
    with Decompressor(unit, device, concatenated) as d:
        return d.decompress(data)


def compress(data, level: int = 9, parallel: int = 10, unit: int = 10000, device: int = 0) -> bytes:
    with Context(level, parallel, unit, device) as ctx:
        return ctx.compress(data)


class OutputStream:
    """Python mirror of the reference OutputStream (OutputStream.hpp:35-241):
    bytes written through write() come out as a .bz2 stream on close()."""

    def __init__(self, out, block_size_multiplier: int = 9, parallel_block_cnt: int = 10, unit: int = 10000):
        if block_size_multiplier < 1 or block_size_multiplier > 9:
            raise ValueError("Invalid block size")
        if parallel_block_cnt < 1:
            raise ValueError("Invalid parallel block count")
        self._out = out
        self._buf = bytearray()
        self._finished = False
        self._ctx = Context(block_size_multiplier, parallel_block_cnt, unit)

    def write(self, value, offset: int = 0, length: int | None = None) -> None:
        if self._finished:
            raise RuntimeError("Write beyond end of stream")
        if isinstance(value, int):
            self._buf.append(value & 0xFF)
        else:
            data = bytes(value)
            if length is None:
                length = len(data) - offset
            self._buf += data[offset: offset + length]

    def close(self) -> None:
        if not self._finished:
            self._finished = True
            self._out.write(self._ctx.compress(bytes(self._buf)))
            self._ctx.close()
