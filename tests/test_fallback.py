"""Totality of the drop-in and the engine's CPU path (the
replacement "must never fail; on any HIP error it falls back"; the
reference function cannot fail, common/crc32c.cc:122-126).

Run here without a GPU, or with MI_CRC32C_FAULT=init in a subprocess: the
total entry points (mi_crc32c, MI_CRC32C_FALLBACK calls, the durable log)
return the oracle's results and every completion is counted in
mi_crc32c_stats; status-returning calls without the flag still fail.  The
multi-device split rule is checked against consus_amd.shard.  The GPU-side
counterparts (fault injected after a live init) are in test_gpu_multi.py."""
import os
import subprocess
import sys

import numpy as np
import pytest

import consus_amd as E
from consus_amd import shard

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code, fault=None):
    env = dict(os.environ)
    if fault:
        env["MI_CRC32C_FAULT"] = fault
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       cwd=REPO, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


FALLBACK_SCRIPT = r"""
import numpy as np, consus_amd as E
from oracle.oracle import Oracle
orc = Oracle()
rng = np.random.default_rng(11)
E.stats_reset()
# the drop-in: check value, chaining, empty input, odd alignments
assert E.crc32c_dropin(0, b"123456789") == 0xE3069283
assert E.crc32c_dropin(0xDEADBEEF, b"") == 0xDEADBEEF
buf = rng.integers(0, 256, 70000, dtype=np.uint8)
for off, n, init in [(0, 1, 0), (3, 31, 7), (5, 4096, 0xFFFFFFFF), (1, 65537, 123)]:
    assert E.crc32c_dropin(init, buf[off:off + n]) == orc.crc32c(init, buf[off:off + n])
# status-returning calls without the flag fail; with it they complete
try:
    E.crc32c_batch(buf, [0], [10])
except E.EngineError as e:
    assert e.status in (E.ENODEV, E.EHIP), e.status
else:
    raise AssertionError("status call without FALLBACK must fail without a GPU engine")
lengths = rng.integers(0, 9000, 500).astype(np.uint32)
offsets = np.zeros(500, dtype=np.uint64)
offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
data = rng.integers(0, 256, int(lengths.sum()) + 1, dtype=np.uint8)
inits = rng.integers(0, 2**32, 500, dtype=np.uint32)
want = orc.batch(data, offsets, lengths, inits)
assert np.array_equal(E.crc32c_batch(data, offsets, lengths, inits, fallback=True), want)
fixed = rng.integers(0, 256, 64 * 4096, dtype=np.uint8)
assert np.array_equal(E.crc32c_fixed(fixed, 4096, 4096, 64, fallback=True),
                      orc.fixed(fixed, 4096, 4096, 64))
# multi-device: the split runs (two ranges named on device 0), each range
# fails on the engine and completes on the CPU path
got = E.crc32c_batch_multi(data, offsets, lengths, inits, devices=[0, 0, 0], shard_min=1,
                           fallback=True)
assert np.array_equal(got, want)
got = E.crc32c_fixed_multi(fixed, 4096, 4096, 64, devices=[0, 0], shard_min=1, fallback=True)
assert np.array_equal(got, orc.fixed(fixed, 4096, 4096, 64))
st = E.stats()
assert st["gpu_calls"] == 0 and st["fallback_calls"] >= 10, st
assert st["last_fallback_status"] in (E.ENODEV, E.EHIP), st
print("FALLBACK OK", st["fallback_calls"], st["fallback_bytes"])
"""


def test_fallback_without_gpu():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present (the GPU variant injects the fault)")
    assert "FALLBACK OK" in _run(FALLBACK_SCRIPT)


def test_fallback_with_injected_init_failure():
    assert "FALLBACK OK" in _run(FALLBACK_SCRIPT, fault="init")


def test_status_calls_still_fail_without_flag():
    out = _run("import consus_amd as E\n"
               "try:\n    E.crc32c(0, b'123456789')\nexcept E.EngineError as e:\n"
               "    print('ERR', e.status)\nelse:\n    print('RAN')\n", fault="init")
    assert "ERR -19" in out, out


def test_bad_arguments_are_not_fallbacks():
    """EINVAL is the caller's error: the CPU path does not paper over it."""
    out = _run("import ctypes as C, consus_amd as E\n"
               "L = E.lib()\n"
               "o = C.c_uint32()\n"
               "print('ST', L.mi_crc32c_buffer(0, None, 5, C.byref(o), E.FLAG_FALLBACK))\n"
               "print('FB', E.stats()['fallback_calls'])\n", fault="init")
    assert "ST -22" in out and "FB 0" in out, out


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 8, 9])
def test_native_split_rule_matches_shard(k):
    rng = np.random.default_rng(k)
    for n in (0, 1, 3, 7, 100, 2500):
        lengths = rng.integers(0, 70000, n).astype(np.uint32)
        if n > 5:
            lengths[rng.integers(0, n, n // 5)] = 0
        assert E.balanced_ranges(lengths, k) == shard.balanced_ranges(lengths, k), (k, n)
    zipf = E.zipf_lengths(0x5EED, 20000)
    assert E.balanced_ranges(zipf, k) == shard.balanced_ranges(zipf, k)
