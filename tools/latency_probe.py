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

# a durable-log flush: 400 frames of 42-1024 B (~215 KB), from pageable and
# from pinned host memory (the log's staging arena is pinned)
lens = rng.integers(42 + 20, 1024 + 20, 400).astype(np.uint32)
offs = np.zeros(lens.size, dtype=np.uint64)
offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
total = int(lens.sum())
pin = E.PinnedBuffer(total)
pin.array[:] = buf[:total]
res = {}
for name, src in (("pageable", buf[:total]), ("pinned", pin.array)):
    for _ in range(20):
        E.crc32c_batch(src, offs, lens)
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        E.crc32c_batch(src, offs, lens)
        ts.append(time.perf_counter() - t0)
    res[name] = sorted(ts)[len(ts) // 2] * 1e6
print(f"400-frame batch ({total} B)  pageable {res['pageable']:7.1f} us   pinned "
      f"{res['pinned']:7.1f} us", flush=True)
