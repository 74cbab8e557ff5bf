"""Per-workgroup timing of the sorted kernel against where it ran (dev tool).

    tools/build_variant.sh stamp -DMI_SORT_STAMP=1
    python tools/wg_hw_probe.py tools/ab/libconsus_crc32c_stamp.so OUT.npz [--mib N] [--launches K]

configs[2] (or its first N MiB of records) through the sorted path with the
stamped build; K times: 20 back-to-back batches, a sync, then the last
batch's per-wave stamps (crc32c_kernels.hip MI_SORT_STAMP) and every
workgroup's HW_ID / XCC_ID register.  Saves stamps[K, 256, 16, 8] (100 MHz
ticks) and hw[K, 256, 2] to OUT.npz for offline analysis: is a slow
workgroup slow because of its share, its XCD, or its physical CU?
"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import consus_amd as E  # noqa: E402
from consus_amd import workload as W  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
E.LIB_PATH = os.path.abspath(args[0])
dest = args[1]
mib = int(sys.argv[sys.argv.index("--mib") + 1]) if "--mib" in sys.argv else 0
K = int(sys.argv[sys.argv.index("--launches") + 1]) if "--launches" in sys.argv else 12
E.init(0)
off, ln, total = W.zipf_records(1 << 20)
if mib:
    n = int(np.searchsorted(np.cumsum(ln, dtype=np.uint64), np.uint64(mib) << np.uint64(20))) + 1
    off, ln = off[:n], ln[:n]
R = len(ln)
hint = int(ln.sum(dtype=np.uint64))
data = E.DeviceBuffer(int(off[-1]) + int(ln[-1]) + 16)
data.fill_splitmix64(W.DATA_SEED)
d_off, d_len, out = E.DeviceBuffer(R * 8), E.DeviceBuffer(R * 4), E.DeviceBuffer(R * 4)
d_off.upload(off)
d_len.upload(ln)
lib = E.lib()
lib.mi_debug_sort_stamps.argtypes = [C.c_void_p, C.c_size_t]
lib.mi_debug_sort_hw.argtypes = [C.c_void_p, C.c_size_t]
for _ in range(60):
    E.device_batch(data, d_off, d_len, R, out, total_bytes=hint, asynchronous=True)
E.sync()
stamps = np.zeros((K, 256, 16, 8), dtype=np.uint64)
hw = np.zeros((K, 256, 2), dtype=np.uint32)
for k in range(K):
    for _ in range(20):
        E.device_batch(data, d_off, d_len, R, out, total_bytes=hint, asynchronous=True)
    E.sync()
    assert lib.mi_debug_sort_stamps(stamps[k].ctypes.data, stamps[k].size) == 0
    assert lib.mi_debug_sort_hw(hw[k].ctypes.data, hw[k].size) == 0
np.savez_compressed(dest, stamps=stamps, hw=hw, records=R, bytes=hint)
st = stamps.astype(np.int64)
us = (st - st[:, :, :, 0].min(axis=(1, 2))[:, None, None, None]) / 100.0
team_end = us[:, :, :, 5].max(axis=2)
print(f"{K} launches of {R} records; team-end spread per launch: "
      + " ".join(f"{x.max() - x.min():.1f}" for x in team_end))
