"""The drop-in boundary from C++ (tools/dropin_check.cc): Consus's own
headers (include/common/crc32c.h, include/txman/durable_log.h) compiled with
g++ and linked against libconsus_crc32c.so alone, as a Consus build would
(INTEGRATION.md section 1).  Built by __graft_entry__.build(); on CPU the
binary must link and fail loudly (no device, no CPU fallback); on the GPU
it checks the check value, chaining, the frame CRC and a durable-log
open/append/wait/replay cycle."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "tools", "dropin_check")


def test_dropin_binary_built_and_linked():
    assert os.path.exists(BIN), "run __graft_entry__.build()"
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True, timeout=60).stdout
    assert "libconsus_crc32c.so" in out and "not found" not in out, out


def test_dropin_fails_loudly_without_device():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "dropin ok" not in r.stdout


@pytest.mark.gpu
def test_dropin_cpp_on_gpu():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "dropin ok" in r.stdout, r.stdout + r.stderr
