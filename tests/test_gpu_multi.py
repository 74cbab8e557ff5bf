"""Multi-device paths on the GPU and the engine's failure
handling with a live device.

  * mi_crc32c_batch[_fixed]_multi: host batches cut into byte-balanced
    ranges, one per named device; on the one-GPU test box the split is forced
    by naming device 0 several times (each range its own worker thread and
    HIP stream), bit-exact against the oracle;
  * the durable log sharding its flushes (MI_CRC32C_DEVICES=0,0);
  * MI_CRC32C_FAULT=compute after a live init: the total entry points still
    return reference results, through the counted CPU path;
  * the N > 1 flows with the engine on every rank: 2 processes on the one GPU
    (tests/_sharded_flows.py), against the reference's golden digests.

Every in-process test here leaves mi_crc32c_stats().fallback_calls at 0
(conftest.py); the fallback runs only in the subprocesses that inject it."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from consus_amd import shard

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def zipf_batch(n, seed=7):
    import consus_amd as E
    lengths = E.zipf_lengths(0x5EED, n, first=seed * 1000)
    offsets = np.zeros(n, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    rng = np.random.default_rng(seed)
    buf = rng.integers(0, 256, int(lengths.sum()) + 64, dtype=np.uint8)
    return buf, offsets, lengths


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0], [0, 0, 0, 0, 0, 0, 0, 0]])
def test_batch_multi_forced_split_parity(engine, oracle, devices):
    buf, off, ln = zipf_batch(20000)
    inits = np.random.default_rng(1).integers(0, 2**32, off.size, dtype=np.uint32)
    before = engine.stats()["sharded_calls"]
    got = engine.crc32c_batch_multi(buf, off, ln, inits, devices=devices, shard_min=1)
    assert np.array_equal(got, oracle.batch(buf, off, ln, inits))
    assert engine.stats()["sharded_calls"] == before + 1
    # unordered records keep their own results
    perm = np.random.default_rng(2).permutation(off.size)
    got = engine.crc32c_batch_multi(buf, off[perm], ln[perm], devices=devices, shard_min=1)
    assert np.array_equal(got, oracle.batch(buf, off[perm], ln[perm]))


def test_batch_multi_threshold_keeps_small_batches_whole(engine, oracle):
    buf, off, ln = zipf_batch(500)  # ~2.3 MB: below one range's worth
    before = engine.stats()["sharded_calls"]
    got = engine.crc32c_batch_multi(buf, off, ln, devices=[0, 0, 0])  # default 4 MiB per range
    assert np.array_equal(got, oracle.batch(buf, off, ln))
    assert engine.stats()["sharded_calls"] == before
    got = engine.crc32c_batch_multi(buf, off, ln)  # every usable device
    assert np.array_equal(got, oracle.batch(buf, off, ln))


def test_fixed_multi_large_host_batch(engine, oracle):
    """256 MiB of 4 KiB records in host memory over 4 ranges (64 MiB each,
    above the default threshold), equal record counts per range."""
    n = 65536
    buf = oracle.fill(n * 4096, 0xC0DE, 0)
    before = engine.stats()["sharded_calls"]
    got = engine.crc32c_fixed_multi(buf, 4096, 4096, n, devices=[0, 0, 0, 0])
    assert engine.stats()["sharded_calls"] == before + 1
    assert np.array_equal(got, oracle.fixed(buf, 4096, 4096, n))
    odd = engine.crc32c_fixed_multi(buf, 4096, 4000, n - 1, devices=[0, 0], shard_min=1)
    assert np.array_equal(odd, oracle.fixed(buf, 4096, 4000, n - 1))


def test_multi_rejects_device_pointers(engine):
    import ctypes as C
    st = engine.lib().mi_crc32c_batch_multi(None, None, None, None, 4, 0, None,
                                            engine.FLAG_DEVICE, None, 0, 0)
    assert st == engine.EINVAL


def _run(code, env_extra, timeout=300):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=REPO,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_fallback_with_compute_fault_on_live_gpu():
    """MI_CRC32C_FAULT=compute: the device initialises, then every compute call
    fails as after a HIP error at run time; the drop-in, FALLBACK batches and
    the multi-device split complete on the CPU path with reference results."""
    from test_fallback import FALLBACK_SCRIPT
    out = _run("import consus_amd as E\nE.init(0)\n" + FALLBACK_SCRIPT,
               {"MI_CRC32C_FAULT": "compute"})
    assert "FALLBACK OK" in out, out


DLOG_SCRIPT = r"""
import numpy as np, consus_amd as E, tempfile, os
from consus_amd.durable_log import DurableLog
E.init(0)
rng = np.random.default_rng(5)
d = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
log = DurableLog(32 << 20, shard_min=1 << 16)
assert log.open(os.path.join(d, "log"))
entries = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes()
           for n in rng.integers(42, 4096, 40000)]
entries[100] = bytes(70 << 20)  # larger than the staging arena: staged on its own
for i, e in enumerate(entries):
    assert log.append(e) == i + 1
x = log.durable()
while x <= len(entries):
    x = log.wait(x)
    assert log.error() == 0
log.close()
assert log.replay() == entries
st = E.stats()
assert st["fallback_calls"] == 0 and st["sharded_calls"] > 0, st
log.destroy()
print("DLOG OK", st["sharded_calls"])
"""


def test_durable_log_shards_flushes():
    out = _run(DLOG_SCRIPT, {"MI_CRC32C_DEVICES": "0,0"})
    assert "DLOG OK" in out, out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_flows_two_ranks_engine_on_each():
    """bench.py's N > 1 flows as a test: 2 ranks on the one GPU, each running
    the engine on its own shard (fixed 2M x 4 KiB, byte-balanced Zipf, one
    slice of an 8 GiB record), checked against the reference's goldens."""
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(REPO, "tests",
                                                                    "_sharded_flows.py")],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      env=env, cwd=REPO))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=240)
            outs.append((p.returncode, o, e))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rc, o, e in outs:
        assert rc == 0, o[-2000:] + e[-2000:]
    line = [x for x in outs[0][1].splitlines() if x.startswith("RESULT ")]
    assert line, outs[0]
    import json
    res = json.loads(line[0][7:])
    assert res["fixed"] and res["zipf"] and res["single"], res
    assert res["fallback_calls"] == [0, 0], res
    assert sum(res["zipf_records_per_rank"]) == 2 << 20
    assert shard.balanced_ranges  # the split rule both ranks used
