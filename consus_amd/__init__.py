"""consus_amd -- MI355X-native CRC-32C engine for Consus's durable-log path.

Python mirror of the reference operator interface (``consus::crc32c``,
common/crc32c.h:40-41) over the C ABI of ``include/consus_crc32c.h``
(``consus_amd/lib/libconsus_crc32c.so``).  Every checksum is computed by the
HIP kernels; if the library is missing, or a gfx950 device is missing, these
calls raise ``EngineError``.  (Only the C drop-in ``mi_crc32c`` /
``consus::crc32c`` and calls made with FLAG_FALLBACK complete on the
engine's CPU path after an engine failure, and every such completion is
counted: ``stats()``.)

    from consus_amd import crc32c, crc32c_batch
    crc32c(0, b"123456789")            # -> 0xE3069283, same as consus::crc32c
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libconsus_crc32c.so")
_DEFAULT_LIB = LIB_PATH
REPO = os.path.dirname(HERE)
HEADERS = [os.path.join(REPO, "include", "consus_crc32c.h"),
           os.path.join(REPO, "include", "consus_durable_log.h")]

OK = 0
EINVAL = -22
ENODEV = -19
ENOMEM = -12
EHIP = -5
ERCCL = -71
FLAG_DEVICE = 0x1
FLAG_ASYNC = 0x2
FLAG_PLANNED = 0x4  # force plan -> chunks -> finalize (no one-launch direct kernel)
FLAG_FALLBACK = 0x8  # host memory: complete on the engine's CPU path if the GPU fails (counted)
MAX_DEVICES = 16
ERANGE = -34
MEMCPY_H2D, MEMCPY_D2H, MEMCPY_D2D = 1, 2, 3


class EngineError(RuntimeError):
    def __init__(self, status: int, what: str, detail: str = ""):
        self.status = status
        super().__init__(f"{what} failed with status {status}: {detail}")


def build() -> None:
    """Compile libconsus_crc32c.so for gfx950 in-tree (hipcc)."""
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(HERE, "csrc")], check=True)


_u8p = C.c_void_p
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)

_SIGS = {
    "mi_crc32c_init": (C.c_int, [C.c_int]),
    "mi_crc32c_strerror": (C.c_char_p, [C.c_int]),
    "mi_crc32c_last_error": (C.c_char_p, []),
    "mi_crc32c_stream": (C.c_void_p, []),
    "mi_crc32c_stream_sync": (C.c_int, []),
    "mi_crc32c": (C.c_uint32, [C.c_uint32, C.c_void_p, C.c_size_t]),
    "mi_crc32c_buffer": (C.c_int, [C.c_uint32, C.c_void_p, C.c_size_t, _u32p, C.c_uint]),
    "mi_crc32c_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                  C.c_uint64, C.c_void_p, C.c_uint]),
    "mi_crc32c_batch_fixed": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                        C.c_size_t, C.c_void_p, C.c_uint]),
    "mi_crc32c_combine": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint64]),
    "mi_crc32c_combine_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                          C.c_void_p, C.c_uint]),
    "mi_crc32c_pipeline_create": (C.c_int, [C.c_size_t, C.c_size_t, C.c_int,
                                            C.POINTER(C.c_void_p)]),
    "mi_crc32c_pipeline_submit": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                            C.POINTER(C.c_uint64)]),
    "mi_crc32c_pipeline_wait": (C.c_int, [C.c_void_p, C.c_uint64]),
    "mi_crc32c_pipeline_destroy": (C.c_int, [C.c_void_p]),
    "mi_dev_malloc": (C.c_int, [C.POINTER(C.c_void_p), C.c_size_t]),
    "mi_dev_free": (C.c_int, [C.c_void_p]),
    "mi_host_malloc_pinned": (C.c_int, [C.POINTER(C.c_void_p), C.c_size_t]),
    "mi_host_free_pinned": (C.c_int, [C.c_void_p]),
    "mi_memcpy": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]),
    "mi_memset": (C.c_int, [C.c_void_p, C.c_int, C.c_size_t]),
    "mi_fill_splitmix64": (C.c_int, [C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint64]),
    "mi_timer_start": (C.c_int, []),
    "mi_timer_stop": (C.c_int, [C.POINTER(C.c_float)]),
    "mi_comm_unique_id": (C.c_int, [C.c_void_p]),
    "mi_comm_init": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "mi_comm_allgather_u32": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p]),
    "mi_comm_destroy": (C.c_int, []),
    "mi_workload_zipf_lengths": (None, [C.c_uint64, C.c_uint64, C.c_size_t, C.c_void_p]),
    "mi_crc32c_device_count": (C.c_int, []),
    "mi_crc32c_stats": (None, [C.c_void_p]),
    "mi_crc32c_stats_reset": (None, []),
    "mi_crc32c_batch_multi": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_size_t, C.c_uint64, C.c_void_p, C.c_uint,
                                        C.c_void_p, C.c_int, C.c_uint64]),
    "mi_crc32c_batch_fixed_multi": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                              C.c_size_t, C.c_void_p, C.c_uint, C.c_void_p,
                                              C.c_int, C.c_uint64]),
    "mi_crc32c_balanced_ranges": (None, [C.c_void_p, C.c_size_t, C.c_int, C.c_uint64,
                                         C.c_void_p]),
    "mi_crc32c_set_gpu_min": (C.c_uint64, [C.c_uint64]),
    "mi_crc32c_gpu_min": (C.c_uint64, []),
    "mi_crc32c_device_pci_bus_id": (C.c_int, [C.c_int, C.c_char_p, C.c_int]),
    "mi_comm_info": (C.c_int, [C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
}


class Stats(C.Structure):
    """mi_crc32c_stats_t (include/consus_crc32c.h)."""
    _fields_ = [("gpu_calls", C.c_uint64), ("fallback_calls", C.c_uint64),
                ("fallback_bytes", C.c_uint64), ("sharded_calls", C.c_uint64),
                ("host_routed_calls", C.c_uint64),
                ("last_fallback_status", C.c_int32),
                ("last_multi_ranges", C.c_int32),
                ("sorted_batches", C.c_uint64),
                ("host_routed_bytes", C.c_uint64),
                ("last_multi_devices", C.c_int32 * MAX_DEVICES),
                ("zero_copy_batches", C.c_uint64),
                ("hint_overflows", C.c_uint64), ("host_batches", C.c_uint64),
                ("host_batch_bytes", C.c_uint64), ("sorted_one_launch", C.c_uint64),
                ("window_batches", C.c_uint64)]

_lib = None


def lib() -> C.CDLL:
    """Load the engine library (raises EngineError if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EngineError(ENODEV, "load", f"{LIB_PATH} missing: run consus_amd.build()")
        L = C.CDLL(LIB_PATH)
        # an A/B build of an earlier round (tools/ab.py, LIB_PATH pointed
        # elsewhere) may lack later entry points; the in-tree library may not
        in_tree = os.path.abspath(LIB_PATH) == os.path.abspath(_DEFAULT_LIB)
        for name, (res, args) in _SIGS.items():
            if not in_tree and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(status: int, what: str) -> None:
    if status != OK:
        detail = (lib().mi_crc32c_last_error() or b"").decode(errors="replace")
        raise EngineError(status, what, detail)


def _np_ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _as_u8(data) -> np.ndarray:
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(data), dtype=np.uint8)
    return np.ascontiguousarray(data).view(np.uint8).reshape(-1)


def init(device: int = 0) -> None:
    _check(lib().mi_crc32c_init(device), "mi_crc32c_init")


# ---- the reference operator -------------------------------------------------
def crc32c(init_crc: int, data, n: int | None = None) -> int:
    """consus::crc32c(init, data, n) (common/crc32c.cc:122-126), on the GPU."""
    a = _as_u8(data)
    n = a.size if n is None else n
    if n > a.size:
        raise ValueError("n exceeds buffer")
    out = C.c_uint32(0)
    _check(lib().mi_crc32c_buffer(init_crc & 0xFFFFFFFF, C.c_void_p(a.ctypes.data), n,
                                  C.byref(out), 0), "mi_crc32c_buffer")
    return int(out.value)


def crc32c_device(buf: "DeviceBuffer", nbytes: int | None = None, init_crc: int = 0,
                  offset: int = 0) -> int:
    """consus::crc32c(init, device bytes [offset, offset + nbytes)) on the GPU."""
    n = buf.nbytes - offset if nbytes is None else nbytes
    out = C.c_uint32(0)
    _check(lib().mi_crc32c_buffer(init_crc & 0xFFFFFFFF, C.c_void_p(buf.ptr + offset), n,
                                  C.byref(out), FLAG_DEVICE), "mi_crc32c_buffer")
    return int(out.value)


def zipf_lengths(seed: int, count: int, first: int = 0) -> np.ndarray:
    """Config-3 record lengths (workload.cc); host-only, no device needed."""
    out = np.zeros(count, dtype=np.uint32)
    lib().mi_workload_zipf_lengths(seed, first, count, C.c_void_p(out.ctypes.data))
    return out


def crc32c_dropin(init_crc: int, data) -> int:
    """The C drop-in mi_crc32c (= consus::crc32c): total, never raises; an
    engine failure completes on the CPU path and shows in stats()."""
    a = _as_u8(data)
    return int(lib().mi_crc32c(init_crc & 0xFFFFFFFF, C.c_void_p(a.ctypes.data), a.size))


def crc32c_batch(buf, offsets, lengths, inits=None, planned: bool = False,
                 fallback: bool = False) -> np.ndarray:
    """Per-record CRCs of host records [buf + off, +len)."""
    a = _as_u8(buf)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    if off.size != ln.size:
        raise ValueError("offsets/lengths size mismatch")
    if off.size and int((off + ln.astype(np.uint64)).max()) > a.size:
        raise ValueError("record outside buffer")
    ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
    out = np.zeros(off.size, dtype=np.uint32)
    _check(lib().mi_crc32c_batch(C.c_void_p(a.ctypes.data), _np_ptr(off), _np_ptr(ln),
                                 _np_ptr(ini), off.size, int(ln.sum(dtype=np.uint64)),
                                 _np_ptr(out), (FLAG_PLANNED if planned else 0) |
                                 (FLAG_FALLBACK if fallback else 0)), "mi_crc32c_batch")
    return out


def crc32c_fixed(buf, stride: int, length: int, count: int, inits=None,
                 fallback: bool = False) -> np.ndarray:
    a = _as_u8(buf)
    if count and (count - 1) * stride + length > a.size:
        raise ValueError("records outside buffer")
    ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
    out = np.zeros(count, dtype=np.uint32)
    _check(lib().mi_crc32c_batch_fixed(C.c_void_p(a.ctypes.data), stride, length, _np_ptr(ini),
                                       count, _np_ptr(out), FLAG_FALLBACK if fallback else 0),
           "mi_crc32c_batch_fixed")
    return out


def stats() -> dict:
    """Process-wide counters: GPU-completed calls, CPU-path fallbacks, size-routed
    host calls, and the device ordinals of the last multi-device call."""
    s = Stats()
    lib().mi_crc32c_stats(C.byref(s))
    d = {f: int(getattr(s, f)) for f, _ in Stats._fields_ if f != "last_multi_devices"}
    d["last_multi_devices"] = [int(x) for x in s.last_multi_devices[:max(s.last_multi_ranges, 0)]]
    return d


def set_gpu_min(nbytes: int) -> int:
    """Single host calls below nbytes run on the CPU path (size routing); 0 =
    every call on the GPU.  Returns the previous threshold."""
    return int(lib().mi_crc32c_set_gpu_min(int(nbytes)))


def gpu_min() -> int:
    return int(lib().mi_crc32c_gpu_min())


def device_pci_bus_id(device: int) -> str:
    buf = C.create_string_buffer(64)
    _check(lib().mi_crc32c_device_pci_bus_id(device, buf, 64), "mi_crc32c_device_pci_bus_id")
    return buf.value.decode()


def stats_reset() -> None:
    lib().mi_crc32c_stats_reset()


def device_count() -> int:
    """Usable gfx950 devices (not initialised)."""
    return int(lib().mi_crc32c_device_count())


def balanced_ranges(lengths, k: int) -> list[tuple[int, int]]:
    """The engine's byte-balanced split rule (mi_crc32c_balanced_ranges)."""
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    bounds = np.zeros(k + 1, dtype=np.uint64)
    lib().mi_crc32c_balanced_ranges(_np_ptr(ln), ln.size, k, int(ln.sum(dtype=np.uint64)),
                                    _np_ptr(bounds))
    return [(int(bounds[r]), int(bounds[r + 1])) for r in range(k)]


def _dev_list(devices):
    if devices is None:
        return None, 0
    d = (C.c_int * len(devices))(*devices)
    return d, len(devices)


def crc32c_batch_multi(buf, offsets, lengths, inits=None, devices=None, shard_min: int = 0,
                       fallback: bool = False, planned: bool = False) -> np.ndarray:
    """Per-record CRCs of a host batch sharded by bytes over several devices
    (mi_crc32c_batch_multi).  devices=None: every usable device."""
    a = _as_u8(buf)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    if off.size != ln.size:
        raise ValueError("offsets/lengths size mismatch")
    if off.size and int((off + ln.astype(np.uint64)).max()) > a.size:
        raise ValueError("record outside buffer")
    ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
    out = np.zeros(off.size, dtype=np.uint32)
    dl, nd = _dev_list(devices)
    flags = (FLAG_FALLBACK if fallback else 0) | (FLAG_PLANNED if planned else 0)
    _check(lib().mi_crc32c_batch_multi(C.c_void_p(a.ctypes.data), _np_ptr(off), _np_ptr(ln),
                                       _np_ptr(ini), off.size, int(ln.sum(dtype=np.uint64)),
                                       _np_ptr(out), flags, dl, nd, shard_min),
           "mi_crc32c_batch_multi")
    return out


def crc32c_fixed_multi(buf, stride: int, length: int, count: int, inits=None, devices=None,
                       shard_min: int = 0, fallback: bool = False) -> np.ndarray:
    a = _as_u8(buf)
    if count and (count - 1) * stride + length > a.size:
        raise ValueError("records outside buffer")
    ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
    out = np.zeros(count, dtype=np.uint32)
    dl, nd = _dev_list(devices)
    _check(lib().mi_crc32c_batch_fixed_multi(C.c_void_p(a.ctypes.data), stride, length,
                                             _np_ptr(ini), count, _np_ptr(out),
                                             FLAG_FALLBACK if fallback else 0, dl, nd, shard_min),
           "mi_crc32c_batch_fixed_multi")
    return out


def combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return int(lib().mi_crc32c_combine(crc_a, crc_b, len_b))


# ---- device-resident buffers ----------------------------------------------------
class DeviceBuffer:
    """A device allocation owned by Python (hipMalloc through the engine)."""

    def __init__(self, nbytes: int):
        p = C.c_void_p(0)
        _check(lib().mi_dev_malloc(C.byref(p), max(int(nbytes), 1)), "mi_dev_malloc")
        self.ptr = int(p.value)
        self.nbytes = int(nbytes)

    def free(self) -> None:
        if self.ptr:
            _check(lib().mi_dev_free(C.c_void_p(self.ptr)), "mi_dev_free")
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def upload(self, arr, offset: int = 0) -> None:
        a = np.ascontiguousarray(arr)
        if offset + a.nbytes > self.nbytes:
            raise ValueError("upload overflows buffer")
        _check(lib().mi_memcpy(C.c_void_p(self.ptr + offset), C.c_void_p(a.ctypes.data), a.nbytes,
                               MEMCPY_H2D), "mi_memcpy")

    def download(self, dtype=np.uint8, count: int | None = None, offset: int = 0) -> np.ndarray:
        dt = np.dtype(dtype)
        n = (self.nbytes - offset) // dt.itemsize if count is None else count
        out = np.empty(n, dtype=dt)
        _check(lib().mi_memcpy(C.c_void_p(out.ctypes.data), C.c_void_p(self.ptr + offset),
                               out.nbytes, MEMCPY_D2H), "mi_memcpy")
        return out

    def fill_splitmix64(self, seed: int, byte_offset: int = 0, nbytes: int | None = None,
                        dst_offset: int = 0) -> None:
        n = self.nbytes - dst_offset if nbytes is None else nbytes
        _check(lib().mi_fill_splitmix64(C.c_void_p(self.ptr + dst_offset), n, seed, byte_offset),
               "mi_fill_splitmix64")

    def memset(self, value: int = 0) -> None:
        _check(lib().mi_memset(C.c_void_p(self.ptr), value, self.nbytes), "mi_memset")


def device_batch_fixed(data: DeviceBuffer, stride: int, length: int, count: int,
                       out: DeviceBuffer, inits: DeviceBuffer | None = None,
                       asynchronous: bool = False, data_offset: int = 0) -> None:
    flags = FLAG_DEVICE | (FLAG_ASYNC if asynchronous else 0)
    _check(lib().mi_crc32c_batch_fixed(C.c_void_p(data.ptr + data_offset), stride, length,
                                       None if inits is None else C.c_void_p(inits.ptr), count,
                                       C.c_void_p(out.ptr), flags), "mi_crc32c_batch_fixed")


def device_batch(data: DeviceBuffer, offsets: DeviceBuffer, lengths: DeviceBuffer, count: int,
                 out: DeviceBuffer, inits: DeviceBuffer | None = None, total_bytes: int = 0,
                 asynchronous: bool = False) -> None:
    flags = FLAG_DEVICE | (FLAG_ASYNC if asynchronous else 0)
    _check(lib().mi_crc32c_batch(C.c_void_p(data.ptr), C.c_void_p(offsets.ptr),
                                 C.c_void_p(lengths.ptr),
                                 None if inits is None else C.c_void_p(inits.ptr), count,
                                 total_bytes, C.c_void_p(out.ptr), flags), "mi_crc32c_batch")


def sync() -> None:
    _check(lib().mi_crc32c_stream_sync(), "mi_crc32c_stream_sync")


def timer_start() -> None:
    _check(lib().mi_timer_start(), "mi_timer_start")


def timer_stop() -> float:
    ms = C.c_float(0)
    _check(lib().mi_timer_stop(C.byref(ms)), "mi_timer_stop")
    return float(ms.value)


# ---- pinned host memory and the streaming pipeline -----------------------------
class PinnedBuffer:
    """Page-locked host memory (hipHostMalloc) exposed as a numpy uint8 array."""

    def __init__(self, nbytes: int):
        p = C.c_void_p(0)
        _check(lib().mi_host_malloc_pinned(C.byref(p), max(int(nbytes), 1)),
               "mi_host_malloc_pinned")
        self.ptr = int(p.value)
        self.nbytes = int(nbytes)
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(self.nbytes, 1)).from_address(self.ptr))

    def free(self) -> None:
        if self.ptr:
            self.array = None
            _check(lib().mi_host_free_pinned(C.c_void_p(self.ptr)), "mi_host_free_pinned")
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Pipeline:
    """H2D -> CRC -> D2H of host segments overlapped over `depth` HIP streams
    (mi_crc32c_pipeline_*).  Results land in `out` at wait(ticket).

    A pageable segment (bytes, numpy array) is copied into pinned staging by
    submit() and may be reused at once.  A PinnedBuffer segment is DMA'd in
    place: do not modify it until wait(ticket) returns (include/consus_crc32c.h).
    """

    def __init__(self, max_segment_bytes: int, max_records: int, depth: int = 2):
        h = C.c_void_p(0)
        _check(lib().mi_crc32c_pipeline_create(max_segment_bytes, max_records, depth,
                                               C.byref(h)), "mi_crc32c_pipeline_create")
        self._h = h
        self._live: dict[int, tuple] = {}

    def submit(self, segment, offsets, lengths, out: np.ndarray, inits=None,
               nbytes: int | None = None) -> int:
        seg = segment if isinstance(segment, PinnedBuffer) else None
        if seg is not None:
            ptr, n = seg.ptr, seg.nbytes if nbytes is None else nbytes
            keep = seg
        else:
            a = _as_u8(segment)
            ptr, n, keep = a.ctypes.data, a.size if nbytes is None else nbytes, a
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        ini = None if inits is None else np.ascontiguousarray(inits, dtype=np.uint32)
        assert out.dtype == np.uint32 and out.size >= off.size and out.flags.c_contiguous
        t = C.c_uint64(0)
        _check(lib().mi_crc32c_pipeline_submit(self._h, C.c_void_p(ptr), n, _np_ptr(off),
                                               _np_ptr(ln), _np_ptr(ini), off.size,
                                               _np_ptr(out), C.byref(t)),
               "mi_crc32c_pipeline_submit")
        self._live[int(t.value)] = (keep, out)
        return int(t.value)

    def wait(self, ticket: int) -> None:
        _check(lib().mi_crc32c_pipeline_wait(self._h, ticket), "mi_crc32c_pipeline_wait")
        self._live.pop(ticket, None)

    def close(self) -> None:
        if self._h:
            _check(lib().mi_crc32c_pipeline_destroy(self._h), "mi_crc32c_pipeline_destroy")
            self._h = None
            self._live.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- RCCL communicator (one process per GPU) --------------------
COMM_ID_BYTES = 128


def comm_unique_id() -> bytes:
    """ncclGetUniqueId on this rank (send it to the others over any control plane)."""
    buf = (C.c_ubyte * COMM_ID_BYTES)()
    _check(lib().mi_comm_unique_id(buf), "mi_comm_unique_id")
    return bytes(buf)


def comm_init(unique_id: bytes, nranks: int, rank: int) -> None:
    if len(unique_id) != COMM_ID_BYTES:
        raise ValueError("unique id must be COMM_ID_BYTES long")
    buf = (C.c_ubyte * COMM_ID_BYTES).from_buffer_copy(unique_id)
    _check(lib().mi_comm_init(buf, nranks, rank), "mi_comm_init")


def comm_allgather_u32(send: DeviceBuffer, count: int, recv: DeviceBuffer) -> None:
    """All-gather `count` u32 per rank into recv (nranks * count u32), synchronous."""
    if send.nbytes < 4 * count:
        raise ValueError("send buffer too small")
    _check(lib().mi_comm_allgather_u32(C.c_void_p(send.ptr), count, C.c_void_p(recv.ptr)),
           "mi_comm_allgather_u32")


def comm_info() -> dict:
    """RCCL's own view of the communicator: ranks (ncclCommCount), this rank,
    and the HIP device it drives."""
    n, r, d = C.c_int(0), C.c_int(0), C.c_int(0)
    _check(lib().mi_comm_info(C.byref(n), C.byref(r), C.byref(d)), "mi_comm_info")
    return {"nranks": int(n.value), "rank": int(r.value), "device": int(d.value)}


def comm_destroy() -> None:
    _check(lib().mi_comm_destroy(), "mi_comm_destroy")
