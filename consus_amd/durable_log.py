"""Python mirror of the batching durable log (include/txman/durable_log.h).

Method names, arguments and return conventions follow consus::durable_log
(txman/durable_log.h:53-93): append() -> recno or -1 (errno via
ctypes.get_errno is not propagated; check error()), durable()/wait() -> the
watermark "every recno < x is durable", replay(f) -> records replayed.
"""
from __future__ import annotations

import ctypes as C

from . import lib as _engine_lib

_REPLAY_CB = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_ubyte), C.c_size_t)
BATCH_CRC_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                           C.c_uint64, C.c_void_p)

_SIGS = {
    "mi_dlog_create": (C.c_void_p, [C.c_size_t]),
    "mi_dlog_create_ex": (C.c_void_p, [C.c_size_t, C.c_int, C.c_uint64]),
    "mi_dlog_create_opts": (C.c_void_p, [C.c_size_t, C.c_int, C.c_uint64, C.c_int64]),
    "mi_dlog_host_flushes": (C.c_uint64, [C.c_void_p]),
    "mi_dlog_set_append_crc_for_testing": (None, [C.c_void_p, C.c_void_p]),
    "mi_dlog_set_external_malloc_failure_for_testing": (None, [C.c_void_p, C.c_int]),
    "mi_dlog_destroy": (None, [C.c_void_p]),
    "mi_dlog_open": (C.c_int, [C.c_void_p, C.c_char_p]),
    "mi_dlog_close": (None, [C.c_void_p]),
    "mi_dlog_append": (C.c_int64, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "mi_dlog_durable": (C.c_int64, [C.c_void_p]),
    "mi_dlog_wait": (C.c_int64, [C.c_void_p, C.c_int64]),
    "mi_dlog_wake": (None, [C.c_void_p]),
    "mi_dlog_error": (C.c_int, [C.c_void_p]),
    "mi_dlog_replay": (C.c_int64, [C.c_void_p, _REPLAY_CB, C.c_void_p]),
    "mi_dlog_flushes": (C.c_uint64, [C.c_void_p]),
    "mi_dlog_frames_flushed": (C.c_uint64, [C.c_void_p]),
    "mi_dlog_external_peak": (C.c_uint64, [C.c_void_p]),
    "mi_dlog_set_batch_crc_for_testing": (None, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "mi_dlog_set_fsync_delay_for_testing": (None, [C.c_void_p, C.c_uint32]),
    "mi_dlog_debug_state": (None, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "mi_dlog_flush_seconds": (None, [C.c_void_p, C.POINTER(C.c_double)]),
    "mi_dlog_scan_file": (C.c_int64, [C.c_char_p, C.POINTER(C.c_uint64), C.c_void_p, C.c_void_p,
                                      C.c_size_t]),
}
_typed = False


def _lib():
    global _typed
    L = _engine_lib()
    if not _typed:
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _typed = True
    return L


class DurableLog:
    def __init__(self, segment_capacity: int = 0, batch_crc=None, gpus: int = 0,
                 shard_min: int = 0, host_batch_max: int = -1):
        """batch_crc: optional C function pointer (mi_dlog_batch_crc) used
        instead of the GPU -- a test hook; must be set before open().
        gpus / shard_min / host_batch_max: consus::durable_log_options
        (devices one flush may shard over, 0 = all usable; per-device share
        threshold, 0 = default; flushes below host_batch_max bytes on the
        CPU, -1 = the measured crossover, 0 = never)."""
        self._h = _lib().mi_dlog_create_opts(segment_capacity, gpus, shard_min, host_batch_max)
        self._keep = batch_crc
        if batch_crc is not None:
            _lib().mi_dlog_set_batch_crc_for_testing(self._h, C.cast(batch_crc, C.c_void_p), None)

    def open(self, path: str) -> bool:
        return bool(_lib().mi_dlog_open(self._h, path.encode()))

    def close(self) -> None:
        _lib().mi_dlog_close(self._h)

    def append(self, entry: bytes) -> int:
        b = bytes(entry)
        return int(_lib().mi_dlog_append(self._h, b, len(b)))

    def durable(self) -> int:
        return int(_lib().mi_dlog_durable(self._h))

    def wait(self, prev_ub: int) -> int:
        return int(_lib().mi_dlog_wait(self._h, prev_ub))

    def wake(self) -> None:
        _lib().mi_dlog_wake(self._h)

    def error(self) -> int:
        return int(_lib().mi_dlog_error(self._h))

    def replay(self) -> list[bytes]:
        out: list[bytes] = []

        def cb(_p, data, n):
            out.append(C.string_at(data, n))
        rc = _lib().mi_dlog_replay(self._h, _REPLAY_CB(cb), None)
        if rc < 0:
            raise OSError("replay failed")
        assert rc == len(out)
        return out

    def flushes(self) -> int:
        return int(_lib().mi_dlog_flushes(self._h))

    def host_flushes(self) -> int:
        """Flushes checksummed on the flush thread's CPU (below host_batch_max)."""
        return int(_lib().mi_dlog_host_flushes(self._h))

    def set_external_malloc_failure_for_testing(self, fail: bool) -> None:
        _lib().mi_dlog_set_external_malloc_failure_for_testing(self._h, int(bool(fail)))

    def frames_flushed(self) -> int:
        return int(_lib().mi_dlog_frames_flushed(self._h))

    def external_peak(self) -> int:
        """Most bytes of oversized frames staged outside the arenas at once."""
        return int(_lib().mi_dlog_external_peak(self._h))

    def flush_seconds(self) -> list:
        """copy wait, frame walk, batch CRC, CRC patch, pwrite, fsync (s)."""
        out = (C.c_double * 6)()
        _lib().mi_dlog_flush_seconds(self._h, out)
        return list(out)

    def set_fsync_delay_for_testing(self, microseconds: int) -> None:
        _lib().mi_dlog_set_fsync_delay_for_testing(self._h, int(microseconds))

    def debug_state(self) -> str:
        """One line of internal state (flush-thread phase, the active
        segment's reservation word, queued jobs, appenders waiting for a
        switch); for watchdogs."""
        buf = C.create_string_buffer(512)
        _lib().mi_dlog_debug_state(self._h, buf, len(buf))
        return buf.value.decode()

    def destroy(self) -> None:
        if self._h:
            _lib().mi_dlog_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def scan_file(path: str, max_frames: int = 0):
    """GPU-verified scan of one segment file -> (valid_frames, valid_bytes)."""
    vb = C.c_uint64(0)
    n = _lib().mi_dlog_scan_file(path.encode(), C.byref(vb), None, None, max_frames)
    if n < 0:
        raise OSError(f"scan of {path} failed")
    return int(n), int(vb.value)
