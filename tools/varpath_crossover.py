"""Piece path vs sorted path crossover (dev tool).

For batches of the configs[2] record stream (Zipf 64 B - 64 KiB, packed)
cut to about 1 .. 256 MiB, times one batch call on each variable-length
path (MI_CRC32C_VARPATH=pieces / sorted; the engine reads it per batch):

  device  device-resident arrays, total_bytes given, launches back to back on
          the engine stream, HIP-event time per batch
  host    pageable host memory, synchronous calls (staging + kernels + D2H),
          median wall time; 'direct' = the engine's own choice (the one-launch
          direct kernel where it applies)

Every result is checked against the first path's CRCs.

    python tools/varpath_crossover.py [--reps N]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import consus_amd as E  # noqa: E402
from consus_amd import workload as W  # noqa: E402

REPS = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 100
SIZES_MIB = [1, 4, 16, 32, 64, 128, 256, 512, 1024, 2048, 0]  # 0 = every record
HOST_MAX_MIB = 256  # host columns only up to here (pageable staging of GBs is slow)

E.init(0)
off_all, ln_all, _ = W.zipf_records(1 << 20)
cum = np.cumsum(ln_all, dtype=np.uint64)
data = E.DeviceBuffer(int(cum[-1]) + 16)
data.fill_splitmix64(W.DATA_SEED)
d_off, d_len = E.DeviceBuffer(8 << 20), E.DeviceBuffer(4 << 20)
out = E.DeviceBuffer(4 << 20)


def warm(seconds=0.3):
    """Back-to-back launches until the GPU clocks have ramped (a cold GPU runs
    short bursts up to 2x slower)."""
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(20):
            E.device_batch_fixed(data, 4096, 4096, 16384, out, asynchronous=True)
        E.sync()


def device_time(n, total, path):
    os.environ["MI_CRC32C_VARPATH"] = path
    for _ in range(3):
        E.device_batch(data, d_off, d_len, n, out, total_bytes=total)
    warm()
    E.timer_start()
    for _ in range(REPS):
        E.device_batch(data, d_off, d_len, n, out, total_bytes=total, asynchronous=True)
    ms = E.timer_stop() / REPS
    return ms, out.download(np.uint32, n)


def host_time(buf, off, ln, path, planned):
    if path:
        os.environ["MI_CRC32C_VARPATH"] = path
    else:
        os.environ.pop("MI_CRC32C_VARPATH", None)
    for _ in range(3):
        E.crc32c_batch(buf, off, ln, planned=planned)
    warm()
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        got = E.crc32c_batch(buf, off, ln, planned=planned)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3, got


print(f"{'MiB':>5} {'records':>8} {'bytes':>11} | device ms: {'pieces':>8} {'sorted':>8} | "
      f"host ms: {'engine':>8} {'pieces':>8} {'sorted':>8}", flush=True)
for mib in SIZES_MIB:
    n = int(np.searchsorted(cum, np.uint64(mib << 20))) + 1 if mib else ln_all.size
    n = min(n, ln_all.size)
    total = int(cum[n - 1])
    d_off.upload(off_all[:n])
    d_len.upload(ln_all[:n])
    dp, cp = device_time(n, total, "pieces")
    ds, cs = device_time(n, total, "sorted")
    assert np.array_equal(cp, cs), f"device paths disagree at {mib} MiB"
    if mib and mib <= HOST_MAX_MIB:
        buf = data.download(np.uint8, total)
        hd, h0 = host_time(buf, off_all[:n], ln_all[:n], None, False)
        hp, h1 = host_time(buf, off_all[:n], ln_all[:n], "pieces", True)
        hs, h2 = host_time(buf, off_all[:n], ln_all[:n], "sorted", True)
        assert np.array_equal(h0, cp) and np.array_equal(h1, cp) and np.array_equal(h2, cp), \
            f"host paths disagree at {mib} MiB"
        host = f"{hd:8.4f} {hp:8.4f} {hs:8.4f}"
    else:
        host = f"{'-':>8} {'-':>8} {'-':>8}"
    print(f"{mib if mib else total >> 20:5d} {n:8d} {total:11d} | {'':11}{dp:8.4f} {ds:8.4f} | {'':9}{host}  "
          f"GB/s {total / dp / 1e6:7.1f} {total / ds / 1e6:7.1f}", flush=True)
os.environ.pop("MI_CRC32C_VARPATH", None)
st = E.stats()
assert st["fallback_calls"] == 0, st
print("stats", st)
