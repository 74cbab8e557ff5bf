"""Latency of one small host call (dev tool): consus::crc32c on host bytes and
a 1-record batch through the planned path, median of 200 calls each."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import consus_amd as E  # noqa: E402

E.init(0)
rng = np.random.default_rng(1)
buf = rng.integers(0, 256, 1 << 21, dtype=np.uint8)
for n in (16, 100, 1024, 4096, 65536, 1 << 20):
    off = np.zeros(1, dtype=np.uint64)
    ln = np.array([n], dtype=np.uint32)
    res = {}
    for name, fn in (("direct", lambda: E.crc32c(0, buf[:n])),
                     ("planned", lambda: E.crc32c_batch(buf, off, ln, planned=True))):
        for _ in range(20):
            fn()
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        res[name] = sorted(ts)[len(ts) // 2] * 1e6
    print(f"n={n:8d}  consus::crc32c {res['direct']:7.1f} us   planned 1-record batch "
          f"{res['planned']:7.1f} us", flush=True)
