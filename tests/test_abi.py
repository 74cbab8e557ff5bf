"""The C-ABI library: loads without a GPU, exports every declared symbol,
its status-returning calls fail loudly when no gfx950 device is present
(only the total drop-in and MI_CRC32C_FALLBACK calls complete on the CPU
path, tests/test_fallback.py), and its host-side operator algebra (combine)
agrees with the oracle."""
import ctypes
import os
import re

import numpy as np
import pytest

import consus_amd as E

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in ("consus_crc32c.h", "consus_durable_log.h"):
        p = os.path.join(REPO, "include", h)
        if not os.path.exists(p):
            continue
        src = re.sub(r"/\*.*?\*/", "", open(p).read(), flags=re.S)
        for m in re.finditer(r"^\s*(?:[A-Za-z_][\w\s\*]*?)\b(mi_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(E.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 29
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_dropin_definition_is_hidden_in_the_executable():
    """consus::crc32c is declared in Consus's hidden namespace (namespace.h:4-5):
    the library exports only the C ABI, and the definition (crc32c_dropin.cc)
    is linked into the executable, as tools/dropin_check shows."""
    lib = ctypes.CDLL(E.LIB_PATH)
    assert not hasattr(lib, "_ZN6consus6crc32cEjPKhm")
    out = __import__("subprocess").run(["nm", "-C", os.path.join(REPO, "tools", "dropin_check")],
                                       capture_output=True, text=True, timeout=60).stdout
    assert "consus::crc32c(unsigned int, unsigned char const*, unsigned long)" in out


def test_combine_host_algebra(oracle):
    rng = np.random.default_rng(5)
    for _ in range(500):
        a, b = (int(x) for x in rng.integers(0, 2**32, 2))
        n = int(rng.integers(0, 1 << 40))
        assert E.combine(a, b, n) == oracle.combine(a, b, n)


def test_no_device_fails_loudly():
    import subprocess
    import sys
    code = ("import consus_amd as E\n"
            "try:\n    E.crc32c(0, b'123456789')\nexcept E.EngineError as e:\n"
            "    print('ERR', e.status)\nelse:\n    print('RAN')\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         cwd=REPO, timeout=120).stdout
    if "RAN" in out:
        pytest.skip("a GPU is present")
    assert "ERR -19" in out, out


def test_cpu_flag_hashes_on_the_engine_cpu_path(oracle):
    """MI_CRC32C_CPU (round 5): a host batch hashed on the engine's CPU path
    by the caller's choice -- no device needed, counted in host_batches and
    host_batch_bytes, never as a fallback; device pointers are refused."""
    lib = E.lib()
    rng = np.random.default_rng(21)
    lengths = rng.integers(0, 3000, 500).astype(np.uint32)
    offsets = np.zeros(500, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1].astype(np.uint64))
    buf = rng.integers(0, 256, int(lengths.sum()) + 8, dtype=np.uint8)
    inits = rng.integers(0, 2**32, 500, dtype=np.uint32)
    out = np.zeros(500, dtype=np.uint32)
    before = E.stats()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    cpu = 0x10
    assert lib.mi_crc32c_batch(p(buf), p(offsets), p(lengths), p(inits), 500, 0, p(out), cpu) == 0
    assert np.array_equal(out, oracle.batch(buf, offsets, lengths, inits))
    st = E.stats()
    assert st["host_batches"] - before["host_batches"] == 1
    assert st["host_batch_bytes"] - before["host_batch_bytes"] == int(lengths.sum())
    assert st["fallback_calls"] == before["fallback_calls"]
    assert lib.mi_crc32c_batch(p(buf), p(offsets), p(lengths), None, 500, 0, p(out), cpu | 0x1) != 0
