"""Sorted-path efficiency probe (dev tool): the same kernel on (a) configs[1]'s
1M x 4 KiB records handed over as a variable-length batch, against the fixed
kernel on the same bytes, and (b) configs[2]'s Zipf batch.  Prints median ms.

python tools/sorted_probe.py [LIB.so]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import consus_amd as E  # noqa: E402
args = [a for a in sys.argv[1:] if not a.startswith("--")]
if args:
    E.LIB_PATH = os.path.abspath(args[0])
from consus_amd import workload as W  # noqa: E402

E.init(0)
os.environ["MI_CRC32C_VARPATH"] = "sorted"


def timed(fn, n=15):
    for _ in range(3):
        fn()
    E.sync()
    t = []
    for _ in range(n):
        E.timer_start()
        fn()
        t.append(E.timer_stop())
    return float(np.median(t)), float(min(t))


R = 1 << 20
L = 4096
data = E.DeviceBuffer(R * L + 16)
data.fill_splitmix64(0xC0DE)
off = np.arange(R, dtype=np.uint64) * np.uint64(L)
ln = np.full(R, L, dtype=np.uint32)
d_off, d_len, out = E.DeviceBuffer(R * 8), E.DeviceBuffer(R * 4), E.DeviceBuffer(R * 4)
d_off.upload(off)
d_len.upload(ln)
fx = timed(lambda: E.device_batch_fixed(data, L, L, R, out, asynchronous=True))
d1 = E.crc32c_device(out, R * 4)
va = timed(lambda: E.device_batch(data, d_off, d_len, R, out, total_bytes=R * L, asynchronous=True))
d2 = E.crc32c_device(out, R * 4)
print(f"4k fixed kernel {fx[0]:.4f} ms (min {fx[1]:.4f}); sorted path {va[0]:.4f} ms (min {va[1]:.4f}) "
      f"{'same' if d1 == d2 else 'DIFFERENT'}")
for b in (data, d_off, d_len, out):
    b.free()
off, ln, total = W.zipf_records(R)
data = E.DeviceBuffer(total + 16)
data.fill_splitmix64(W.DATA_SEED)
d_off, d_len, out = E.DeviceBuffer(R * 8), E.DeviceBuffer(R * 4), E.DeviceBuffer(R * 4)
d_off.upload(off)
d_len.upload(ln)
z = timed(lambda: E.device_batch(data, d_off, d_len, R, out, total_bytes=total, asynchronous=True))
print(f"zipf sorted path {z[0]:.4f} ms (min {z[1]:.4f}) {total / z[0] / 1e6:.1f} GB/s")
