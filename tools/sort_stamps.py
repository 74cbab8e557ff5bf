"""Where a sorted-path batch's time goes, wave by wave (dev tool).

    tools/build_variant.sh stamp -DMI_SORT_STAMP=1
    python tools/sort_stamps.py tools/ab/libconsus_crc32c_stamp.so [--mib N]

Runs the configs[2] batch (or its first N MiB of records) through the sorted
path with the stamped build (crc32c_kernels.hip, MI_SORT_STAMP: lane 0 of every
wave stores s_memrealtime, 100 MHz, at 8 points), then prints, in us after
the kernel's first wave started: the median wave's time at each point, the
spread of the workgroups' ends, and per XCD group (workgroup % 8) the median
workgroup end.  Stamps are from the last of several back-to-back batches.
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
mib = int(sys.argv[sys.argv.index("--mib") + 1]) if "--mib" in sys.argv else 0
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
for _ in range(int(os.environ.get("STAMP_WARM", "60"))):
    E.device_batch(data, d_off, d_len, R, out, total_bytes=hint, asynchronous=True)
E.sync()
lib = E.lib()
lib.mi_debug_sort_stamps.argtypes = [C.c_void_p, C.c_size_t]
st = np.zeros(256 * 16 * 8, dtype=np.uint64)
assert lib.mi_debug_sort_stamps(st.ctypes.data, st.size) == 0
st = st.reshape(256, 16, 8).astype(np.int64)
t0 = st[:, :, 0].min()
us = (st - t0) / 100.0  # 100 MHz -> us
names = ["entry", "blocks found", "resolved", "binned", "first group", "teams done",
         "lanes done", "finish done"]
last = 7 if (st[:, :, 7] > 0).all() else 6
print(f"records {R}, bytes {hint}; us after the first wave's entry (median wave / min / max)")
for k in range(last + 1):
    v = us[:, :, k]
    print(f"  {names[k]:13s} {np.median(v):8.2f} {v.min():8.2f} {v.max():8.2f}")
wg_end = us[:, :, last].max(axis=1)
team_end = us[:, :, 5].max(axis=1)
print(f"workgroup end: min {wg_end.min():.2f} median {np.median(wg_end):.2f} max {wg_end.max():.2f}")
print(f"team groups end (per workgroup, last wave): min {team_end.min():.2f} "
      f"median {np.median(team_end):.2f} max {team_end.max():.2f}")
lane_t = (us[:, :, 6] - us[:, :, 5])
print(f"lane phase per wave: median {np.median(lane_t):.2f} max {lane_t.max():.2f}")
if last == 7:
    fin = us[:, :, 7].max(axis=1) - us[:, :, 6].max(axis=1)
    print(f"finish pass per workgroup (after its last lane wave): median {np.median(fin):.2f} "
          f"max {fin.max():.2f}")
# within one workgroup: how far apart its waves finish their team groups
# (each wave takes groups from the workgroup's LDS counter, largest first)
intra = us[:, :, 5].max(axis=1) - us[:, :, 5].min(axis=1)
idle = (us[:, :, 5].max(axis=1)[:, None] - us[:, :, 5]).mean(axis=1)
print(f"team-phase end spread within a workgroup (last - first wave): median {np.median(intra):.2f} "
      f"max {intra.max():.2f}; mean wave wait for its workgroup's last wave: median {np.median(idle):.2f} "
      f"max {idle.max():.2f}")
print("per XCD group (workgroup % 8): median workgroup end " +
      " ".join(f"{np.median(wg_end[x::8]):.1f}" for x in range(8)))


def ends_of_next(k):
    """Team-phase ends per workgroup (us after that launch's start) of k more
    single batches, each read back after its own sync."""
    res = []
    for _ in range(k):
        E.device_batch(data, d_off, d_len, R, out, total_bytes=hint, asynchronous=True)
        E.sync()
        s2 = np.zeros(256 * 16 * 8, dtype=np.uint64)
        assert lib.mi_debug_sort_stamps(s2.ctypes.data, s2.size) == 0
        s2 = s2.reshape(256, 16, 8).astype(np.int64)
        u2 = (s2 - s2[:, :, 0].min()) / 100.0
        res.append(u2[:, :, 5].max(axis=1))
    return res


# Is a workgroup's speed a property of where it runs (the same workgroups slow
# launch after launch), or noise?  Correlation of the per-workgroup team-phase
# ends of consecutive launches (the shares are the same batch's).
if "--repeat" in sys.argv:
    k = int(sys.argv[sys.argv.index("--repeat") + 1])
    ends = [team_end] + ends_of_next(k)
    m = np.array(ends)
    dev = m - m.mean(axis=1, keepdims=True)
    c = np.corrcoef(dev)
    print(f"team-end spread per launch (max - min, us): " + " ".join(f"{x.max() - x.min():.1f}" for x in m))
    print(f"correlation of per-workgroup team ends between launches: min {c[np.triu_indices(len(m), 1)].min():.3f} "
          f"mean {c[np.triu_indices(len(m), 1)].mean():.3f}")
    avg = dev.mean(axis=0)
    print(f"per-workgroup mean deviation over launches: sd {avg.std():.2f} us, per-launch residual sd "
          f"{(dev - avg).std():.2f} us")
    print("per XCD group mean deviation: " + " ".join(f"{avg[x::8].mean():+.1f}" for x in range(8)))
