"""Cost of the multi-device split (mi_crc32c_batch_fixed_multi) on one GPU.

For host batches of 4 KiB records (pageable memory) of 1-512 MiB: the time
of one call on one device (devices=[0]) and of the same call forced into 2
ranges (devices=[0, 0], shard_min=1: two worker threads, two streams, both
ranges over the same PCIe link).  On one GPU the split cannot be faster --
the link is shared -- so the difference is what a split costs; the one-device
rate is what a second device's link would add.  Median of 7 calls each.
Output: one line per size (profiles/r02_shard_overhead.txt)."""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
import consus_amd as E  # noqa: E402

E.init(0)
print("# host batch of 4 KiB records, pageable memory; ms per call (median of 7)")
print("# size_MiB  one_device_ms  GB/s   split_2_on_one_device_ms  split_cost_ms")
for mib in (1, 4, 16, 64, 256, 512):
    n = mib * 256
    buf = np.random.default_rng(mib).integers(0, 256, n * 4096, dtype=np.uint8)
    want = E.crc32c_fixed_multi(buf, 4096, 4096, n, devices=[0])
    res = {}
    for name, devs in (("one", [0]), ("split", [0, 0])):
        ts = []
        for _ in range(7):
            t0 = time.perf_counter()
            got = E.crc32c_fixed_multi(buf, 4096, 4096, n, devices=devs, shard_min=1)
            ts.append(time.perf_counter() - t0)
            assert np.array_equal(got, want)
        res[name] = float(np.median(ts)) * 1e3
    print(f"{mib:8d}  {res['one']:12.3f}  {n * 4096 / res['one'] / 1e6:6.1f}  "
          f"{res['split']:22.3f}  {res['split'] - res['one']:12.3f}", flush=True)
print("stats", E.stats())
