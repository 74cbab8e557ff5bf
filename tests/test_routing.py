"""Size routing at the drop-in boundary (include/
consus_crc32c.h mi_crc32c_set_gpu_min): single host calls below the GPU
threshold are answered by the engine's CPU path without a GPU round trip and
counted as host_routed_calls -- never as fallbacks; larger calls, batches and
device buffers go to the engine.  CPU-runnable: each case runs in a
subprocess with its own MI_CRC32C_GPU_MIN (the suite itself runs with 0)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r"""
import json, sys
import numpy as np
sys.path.insert(0, %r)
import consus_amd as E
from oracle.oracle import Oracle
orc = Oracle()
rng = np.random.default_rng(7)
res = {"gpu_min_at_load": E.gpu_min()}
small = rng.integers(0, 256, 100, dtype=np.uint8)
res["small_ok"] = E.crc32c_dropin(0x1234, small) == orc.crc32c(0x1234, small)
res["after_small"] = E.stats()
try:
    res["buffer_ok"] = E.crc32c(7, small[:50]) == orc.crc32c(7, small[:50])
except E.EngineError as e:  # status-returning call, engine without a device
    res["buffer_ok"] = e.status
res["after_buffer"] = E.stats()
big = rng.integers(0, 256, 10000, dtype=np.uint8)
res["big_ok"] = E.crc32c_dropin(0, big) == orc.crc32c(0, big)
res["after_big"] = E.stats()
res["prev"] = E.set_gpu_min(0)
res["now"] = E.gpu_min()
res["zero_ok"] = E.crc32c_dropin(0, small) == orc.crc32c(0, small)
res["after_zero"] = E.stats()
print(json.dumps(res))
""" % REPO


def run(env_min):
    env = dict(os.environ)
    env["MI_CRC32C_GPU_MIN"] = str(env_min)
    out = subprocess.run([sys.executable, "-c", CODE], capture_output=True, text=True, cwd=REPO,
                         env=env, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def gpu_present():
    import consus_amd as E
    return E.device_count() > 0


def test_small_calls_are_routed_and_counted_not_fallbacks():
    r = run(4096)
    assert r["gpu_min_at_load"] == 4096
    assert r["small_ok"] and r["buffer_ok"] and r["big_ok"] and r["zero_ok"]
    s = r["after_small"]
    assert s["host_routed_calls"] == 1 and s["host_routed_bytes"] == 100
    assert s["fallback_calls"] == 0 and s["gpu_calls"] == 0
    s = r["after_buffer"]
    assert s["host_routed_calls"] == 2 and s["host_routed_bytes"] == 150
    # 10,000 B >= 4096: the engine; without a GPU that is a counted fallback
    s = r["after_big"]
    assert s["host_routed_calls"] == 2
    if gpu_present():
        assert s["gpu_calls"] == 1 and s["fallback_calls"] == 0
    else:
        assert s["fallback_calls"] == 1 and s["gpu_calls"] == 0
    # threshold 0 at run time: nothing is routed any more
    assert r["prev"] == 4096 and r["now"] == 0
    assert r["after_zero"]["host_routed_calls"] == 2


def test_threshold_zero_routes_nothing():
    r = run(0)
    assert r["small_ok"] and r["big_ok"]
    assert r["buffer_ok"] is True or (r["buffer_ok"] == -19 and not gpu_present())
    assert r["after_big"]["host_routed_calls"] == 0


def test_default_threshold_is_the_measured_crossover():
    code = "import consus_amd as E; print(E.gpu_min())"
    env = {k: v for k, v in os.environ.items() if k != "MI_CRC32C_GPU_MIN"}
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=REPO,
                         env=env, timeout=120)
    assert out.returncode == 0, out.stderr
    assert int(out.stdout.strip()) > 0
