"""The drop-in boundary from C++ (tools/dropin_check.cc): Consus's own
headers (include/common/crc32c.h, include/txman/durable_log.h) compiled with
g++ and linked against libconsus_crc32c.so alone, as a Consus build would
(INTEGRATION.md section 1).  Built by __graft_entry__.build().  It checks the
check value, chaining, the frame CRC and a durable-log open/append/wait/
replay cycle.  Without a device (here) every check still passes -- the drop-in
is total, as common/crc32c.cc:122-126 is -- and the binary reports CPU-path
fallbacks; on the GPU it must report none (the HIP kernels did the work)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "tools", "dropin_check")


def test_dropin_binary_built_and_linked():
    assert os.path.exists(BIN), "run __graft_entry__.build()"
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True, timeout=60).stdout
    assert "libconsus_crc32c.so" in out and "not found" not in out, out


def _counts(out):
    kv = dict(t.split("=") for t in out.split() if "=" in t)
    return int(kv["gpu_calls"]), int(kv["fallback_calls"])


def test_dropin_total_without_device():
    """No GPU: same answers through the engine's CPU path, every one counted."""
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "dropin ok" in r.stdout, r.stdout + r.stderr
    gpu, fb = _counts(r.stdout)
    assert gpu == 0 and fb > 0


def test_dropin_total_with_injected_init_failure():
    """MI_CRC32C_FAULT=init: the engine refuses every device (as after a
    failed initialisation); the C++ drop-in and the durable log still return
    reference results, through the counted CPU path."""
    env = dict(os.environ, MI_CRC32C_FAULT="init")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "dropin ok" in r.stdout, r.stdout + r.stderr
    gpu, fb = _counts(r.stdout)
    assert gpu == 0 and fb > 0


@pytest.mark.gpu
def test_dropin_cpp_on_gpu():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "dropin ok" in r.stdout, r.stdout + r.stderr
    gpu, fb = _counts(r.stdout)
    assert gpu > 0 and fb == 0, r.stdout


@pytest.mark.gpu
def test_dropin_cpp_total_on_gpu_with_compute_fault():
    """MI_CRC32C_FAULT=compute on a live GPU: the device initialises, every
    compute call then fails as after a HIP error at run time; the drop-in and
    the log complete on the CPU path with reference results."""
    env = dict(os.environ, MI_CRC32C_FAULT="compute")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "dropin ok" in r.stdout, r.stdout + r.stderr
    gpu, fb = _counts(r.stdout)
    assert gpu == 0 and fb > 0
