"""ctypes loader for the CPU checkers (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
may import this module.  The product package ``consus_amd`` never does.

Two libraries:
  * ``liboracle.so``             -- the C restatement (crc32c_oracle.c)
  * ``_ref/libref_crc32c.so``    -- the reference common/crc32c.cc compiled
                                    unmodified (ref_driver.cc); optional.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_crc32c.so")

_u8p = C.POINTER(C.c_uint8)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)


def build() -> None:
    """Build liboracle.so (and _ref when /root/reference is present)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _ptr(a, t):
    if a is None:
        return None
    return a.ctypes.data_as(t)


def _as_u8(data):
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(data), dtype=np.uint8)
    return np.ascontiguousarray(data).view(np.uint8).reshape(-1)


class _Lib:
    def __init__(self, path: str):
        self.path = path
        self.lib = C.CDLL(path)


class Oracle(_Lib):
    """The C restatement."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build()
        super().__init__(path)
        L = self.lib
        for name in ("oracle_crc32c", "oracle_crc32c_bitwise", "oracle_crc32c_sb8",
                     "oracle_crc32c_sse42"):
            f = getattr(L, name)
            f.restype = C.c_uint32
            f.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
        L.oracle_has_sse42.restype = C.c_int
        L.oracle_shift.restype = C.c_uint32
        L.oracle_shift.argtypes = [C.c_uint32, C.c_uint64]
        L.oracle_crc32c_combine.restype = C.c_uint32
        L.oracle_crc32c_combine.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
        L.oracle_crc32c_batch.restype = None
        L.oracle_crc32c_batch.argtypes = [C.c_void_p, _u64p, _u32p, _u32p, C.c_size_t, _u32p,
                                          C.c_int]
        L.oracle_crc32c_fixed.restype = None
        L.oracle_crc32c_fixed.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, _u32p, C.c_size_t,
                                          _u32p, C.c_int]
        L.oracle_digest.restype = C.c_uint32
        L.oracle_digest.argtypes = [_u32p, C.c_size_t, _u32p]
        L.oracle_fill.restype = None
        L.oracle_fill.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint64]
        L.oracle_tables.restype = None
        L.oracle_tables.argtypes = [_u32p]

    # single buffer ---------------------------------------------------------
    def crc32c(self, init: int, data, n: int | None = None, offset: int = 0,
               impl: str = "api") -> int:
        a = _as_u8(data)
        n = a.size - offset if n is None else n
        f = {"api": self.lib.oracle_crc32c, "bitwise": self.lib.oracle_crc32c_bitwise,
             "sb8": self.lib.oracle_crc32c_sb8, "sse42": self.lib.oracle_crc32c_sse42}[impl]
        return int(f(init & 0xFFFFFFFF, a.ctypes.data + offset, n))

    def shift(self, s: int, nbytes: int) -> int:
        return int(self.lib.oracle_shift(s & 0xFFFFFFFF, nbytes))

    def combine(self, a: int, b: int, len_b: int) -> int:
        return int(self.lib.oracle_crc32c_combine(a, b, len_b))

    # batches ---------------------------------------------------------------
    def batch(self, buf, offsets, lengths, inits=None, threads: int = 8) -> np.ndarray:
        a = _as_u8(buf)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
        out = np.zeros(off.size, dtype=np.uint32)
        self.lib.oracle_crc32c_batch(a.ctypes.data, _ptr(off, _u64p), _ptr(ln, _u32p),
                                     _ptr(ini, _u32p), off.size, _ptr(out, _u32p), threads)
        return out

    def fixed(self, buf, stride: int, length: int, count: int, inits=None,
              threads: int = 8) -> np.ndarray:
        a = _as_u8(buf)
        assert count == 0 or (count - 1) * stride + length <= a.size
        ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
        out = np.zeros(count, dtype=np.uint32)
        self.lib.oracle_crc32c_fixed(a.ctypes.data, stride, length, _ptr(ini, _u32p), count,
                                     _ptr(out, _u32p), threads)
        return out

    def digest(self, crcs) -> tuple[int, int]:
        c = np.ascontiguousarray(crcs, dtype=np.uint32)
        x = C.c_uint32(0)
        d = self.lib.oracle_digest(_ptr(c, _u32p), c.size, C.byref(x))
        return int(d), int(x.value)

    def fill(self, nbytes: int, seed: int, byte_offset: int = 0) -> np.ndarray:
        out = np.empty(nbytes, dtype=np.uint8)
        self.lib.oracle_fill(out.ctypes.data, nbytes, seed, byte_offset)
        return out

    def tables(self) -> np.ndarray:
        out = np.zeros((16, 256), dtype=np.uint32)
        self.lib.oracle_tables(_ptr(out, _u32p))
        return out


class Reference(_Lib):
    """The reference common/crc32c.cc compiled unmodified (oracle/_ref)."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        super().__init__(path)
        L = self.lib
        for name in ("ref_crc32c", "ref_crc32c_sw", "ref_crc32c_hw"):
            f = getattr(L, name)
            f.restype = C.c_uint32
            f.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
        L.ref_dispatch_is_sse42.restype = C.c_int
        L.ref_tables.restype = None
        L.ref_tables.argtypes = [_u32p]
        L.ref_crc32c_fixed_mt.restype = None
        L.ref_crc32c_fixed_mt.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, _u32p, C.c_size_t,
                                          _u32p, C.c_int]
        L.ref_crc32c_batch_mt.restype = None
        L.ref_crc32c_batch_mt.argtypes = [C.c_void_p, _u64p, _u32p, _u32p, C.c_size_t, _u32p,
                                          C.c_int]
        L.ref_crc32c_splitmix_var.restype = None
        L.ref_crc32c_splitmix_var.argtypes = [C.c_uint64, _u64p, _u32p, C.c_size_t, _u32p,
                                              C.c_int]
        L.ref_crc32c_splitmix_fixed.restype = None
        L.ref_crc32c_splitmix_fixed.argtypes = [C.c_uint64, C.c_size_t, C.c_uint64, C.c_size_t,
                                                _u32p, C.c_int]

    def splitmix_var(self, seed: int, offsets, lengths, threads: int = 8) -> np.ndarray:
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        out = np.zeros(off.size, dtype=np.uint32)
        self.lib.ref_crc32c_splitmix_var(seed, _ptr(off, _u64p), _ptr(ln, _u32p), off.size,
                                         _ptr(out, _u32p), threads)
        return out

    def crc32c(self, init: int, data, n: int | None = None, offset: int = 0,
               impl: str = "api") -> int:
        a = _as_u8(data)
        n = a.size - offset if n is None else n
        f = {"api": self.lib.ref_crc32c, "sw": self.lib.ref_crc32c_sw,
             "hw": self.lib.ref_crc32c_hw}[impl]
        return int(f(init & 0xFFFFFFFF, a.ctypes.data + offset, n))

    def tables(self) -> np.ndarray:
        out = np.zeros((8, 256), dtype=np.uint32)
        self.lib.ref_tables(_ptr(out, _u32p))
        return out

    def fixed(self, buf, stride: int, length: int, count: int, inits=None,
              threads: int = 1) -> np.ndarray:
        a = _as_u8(buf)
        assert count == 0 or (count - 1) * stride + length <= a.size
        ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
        out = np.zeros(count, dtype=np.uint32)
        self.lib.ref_crc32c_fixed_mt(a.ctypes.data, stride, length, _ptr(ini, _u32p), count,
                                     _ptr(out, _u32p), threads)
        return out

    def batch(self, buf, offsets, lengths, inits=None, threads: int = 1) -> np.ndarray:
        a = _as_u8(buf)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
        out = np.zeros(off.size, dtype=np.uint32)
        self.lib.ref_crc32c_batch_mt(a.ctypes.data, _ptr(off, _u64p), _ptr(ln, _u32p),
                                     _ptr(ini, _u32p), off.size, _ptr(out, _u32p), threads)
        return out

    def splitmix_stream(self, seed: int, byte_off: int, nbytes: int) -> int:
        """consus::crc32c(0, stream bytes [byte_off, +nbytes)), chained in 4 MiB pieces."""
        f = self.lib.ref_crc32c_splitmix_stream
        f.restype, f.argtypes = C.c_uint32, [C.c_uint64, C.c_uint64, C.c_uint64]
        return int(f(seed, byte_off, nbytes))

    def splitmix_fixed(self, seed: int, rec_len: int, first_rec: int, count: int,
                       threads: int = 8) -> np.ndarray:
        out = np.zeros(count, dtype=np.uint32)
        self.lib.ref_crc32c_splitmix_fixed(seed, rec_len, first_rec, count, _ptr(out, _u32p),
                                           threads)
        return out


def reference_available() -> bool:
    return os.path.exists(REF_SO)
