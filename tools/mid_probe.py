"""Mid-size device batches (dev tool, VERDICT r3 Next 4): the configs[2]
record stream cut to N MiB, timed per batch on the chosen variable-length path
(MI_CRC32C_VARPATH, default: the engine's choice), HIP events over R
back-to-back batches after a clock warm-up; checked against the oracle.

    python tools/mid_probe.py [--mib 16,64,256] [--reps 200] [--path pieces|sorted|mid]
                              [--uniform LO,HI]

--uniform LO,HI replaces the configs[2] lengths with uniform LO..HI-byte
records packed back to back (durable-log-like entries: 42,1024).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import consus_amd as E  # noqa: E402
from consus_amd import workload as W  # noqa: E402


def arg(name, default):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


SIZES = [int(x) for x in arg("--mib", "1,4,16,64,256").split(",")]
if "--lib" in sys.argv:
    E.LIB_PATH = os.path.abspath(arg("--lib", ""))
REPS = int(arg("--reps", "200"))
PATH = arg("--path", "")
if PATH:
    os.environ["MI_CRC32C_VARPATH"] = PATH

E.init(0)
off_all, ln_all, _ = W.zipf_records(1 << 20)
if "--uniform" in sys.argv:
    lo, hi = (int(x) for x in arg("--uniform", "42,1024").split(","))
    ln_all = np.random.default_rng(7).integers(lo, hi + 1, ln_all.size).astype(np.uint32)
    off_all = np.zeros(ln_all.size, dtype=np.uint64)
    off_all[1:] = np.cumsum(ln_all[:-1], dtype=np.uint64)
cum = np.cumsum(ln_all, dtype=np.uint64)
data = E.DeviceBuffer(int(cum[-1]) + 16)
data.fill_splitmix64(W.DATA_SEED)
d_off, d_len = E.DeviceBuffer(8 << 20), E.DeviceBuffer(4 << 20)
out = E.DeviceBuffer(4 << 20)
host = None


def warm(seconds=0.3):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(20):
            E.device_batch_fixed(data, 4096, 4096, 16384, out, asynchronous=True)
        E.sync()


TAG = os.path.basename(arg("--lib", "")) or (PATH or "engine")
print(f"path={PATH or 'engine'}  {'MiB':>5} {'records':>8} {'bytes':>11}  ms/batch   GB/s   check",
      flush=True)
for mib in SIZES:
    n = int(np.searchsorted(cum, np.uint64(mib) << np.uint64(20))) + 1 if mib else len(ln_all)
    n = min(n, len(ln_all))
    off, ln = off_all[:n], ln_all[:n]
    total = int(ln.sum(dtype=np.uint64))
    d_off.upload(off)
    d_len.upload(ln)
    for _ in range(3):
        E.device_batch(data, d_off, d_len, n, out, total_bytes=total)
    got = out.download(np.uint32, n)
    if host is None:
        host = data.download(np.uint8, int(cum[-1]))
    from oracle import oracle as O  # checker only
    want = O.Oracle().batch(host, off, ln)
    ok = np.array_equal(got, want)
    warm()
    E.timer_start()
    for _ in range(REPS):
        E.device_batch(data, d_off, d_len, n, out, total_bytes=total, asynchronous=True)
    ms = E.timer_stop() / REPS
    print(f"{TAG}  {mib:5d} {n:8d} {total:11d}  {ms:8.4f} {total / ms / 1e6:7.1f}   "
          f"{'OK' if ok else 'MISMATCH'}", flush=True)
