"""pytest configuration: the `gpu` marker and shared fixtures.

`-m "not gpu"` runs here (no GPU): oracle vs golden vectors, host logic, the
C-ABI library loading/exports.  `-m gpu` runs on the MI355X box: parity of
the HIP kernels against the oracle through the C ABI.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

# Size routing off (include/consus_crc32c.h, mi_crc32c_set_gpu_min): every
# call of the suite, and of the tools it starts, goes to the GPU engine, so
# the GPU tests certify the HIP kernels.  tests/test_routing.py turns it on
# where it tests it.
os.environ["MI_CRC32C_GPU_MIN"] = "0"
# Likewise the durable log's flush routing (durable_log_options::host_batch_max):
# every flush of the suite is checksummed by the GPU batch;
# tests/test_durable_log.py::test_small_flushes_route_to_the_cpu turns it on.
os.environ["MI_DLOG_HOST_BATCH_MAX"] = "0"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def reference():
    from oracle.oracle import Reference, reference_available
    if not reference_available():
        pytest.skip("oracle/_ref/libref_crc32c.so not built")
    return Reference()


@pytest.fixture(autouse=True)
def _gpu_path_certified(request):
    """Every GPU test certifies the HIP kernels: the engine's CPU path must not
    have run in this process, neither after a failure (fallback_calls) nor by
    size routing (host_routed_calls).  Tests that exercise either on purpose
    do it in a subprocess."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import consus_amd
    st = consus_amd.stats()
    assert st["fallback_calls"] == 0, f"CPU-path fallback ran during a GPU test: {st}"
    assert st["host_routed_calls"] == 0, f"size-routed CPU call during a GPU test: {st}"


@pytest.fixture(scope="session")
def engine():
    import consus_amd
    consus_amd.init(0)
    return consus_amd
