"""Per-wave timeline of one configs[2] batch through the sorted path (dev
tool, needs a MI_SORT_STAMP=1 build): prologue end and last-group end of every
wave relative to the earliest wave start, in microseconds.

python tools/sorted_stamps.py LIB.so
"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import consus_amd as E  # noqa: E402
E.LIB_PATH = os.path.abspath(sys.argv[1])
from consus_amd import workload as W  # noqa: E402

E.init(0)
os.environ["MI_CRC32C_VARPATH"] = "sorted"
R = 1 << 20
off, ln, total = W.zipf_records(R)
if os.environ.get("ZIPF_KEEP_BELOW"):  # one length class only (tools/zipf_probe.py)
    ln = np.where(ln < int(os.environ["ZIPF_KEEP_BELOW"]), ln, 0).astype(ln.dtype)
data = E.DeviceBuffer(total + 16)
data.fill_splitmix64(W.DATA_SEED)
d_off, d_len, out = E.DeviceBuffer(R * 8), E.DeviceBuffer(R * 4), E.DeviceBuffer(R * 4)
d_off.upload(off)
d_len.upload(ln)
for _ in range(4):
    E.device_batch(data, d_off, d_len, R, out, total_bytes=total)
E.lib().mi_dev_sorted_stamps.restype = C.c_void_p
ptr = E.lib().mi_dev_sorted_stamps()
buf = E.DeviceBuffer.__new__(E.DeviceBuffer)
buf.ptr, buf.nbytes = ptr, 4096 * 64
st = buf.download(np.uint64, 4096 * 8).reshape(4096, 8).astype(np.int64)
buf.ptr = 0
t0 = st[:, 0].min()
pro = (st[:, 1] - t0) / 100.0
end = (st[:, 2] - t0) / 100.0
q = lambda a: " ".join(f"{p}%={np.percentile(a, p):.1f}" for p in (0, 1, 10, 50, 90, 99, 100))
print("start   ", q((st[:, 0] - t0) / 100.0))
MODE2 = os.environ.get("STAMP_MODE") == "2"  # a MI_SORT_STAMP=2 build
for i, name in ((3, "staged"), (4, "blocks found"), (5, "resolved"),
                (6, "first <= 8 rows" if MODE2 else "pass 1"), (7, "first <= 2 rows" if MODE2 else "allocated"),
                (1, "pass 2 = prologue")):
    v = st[:, i][st[:, i] > 0] if MODE2 and i in (6, 7) else st[:, i]
    print(f"{name:18s}", q((v - t0) / 100.0), f"({v.size} waves)" if MODE2 and i in (6, 7) else "")
print("end     ", q(end))
wg_end = end.reshape(256, 16).max(axis=1)
wg_min = end.reshape(256, 16).min(axis=1)
print("WG end (max wave)", q(wg_end))
print("WG spread (last - first wave end)", q(wg_end - wg_min))
# per-workgroup analysis: the workgroup's cost share under the kernel's model
# (rows + 2 per item, records < 4 B free) against its end time
L = ln.astype(np.int64)
a = off.astype(np.int64)  # base offset 0 is 256-aligned, so alignment = offset
rows = ((a + L + 127) // 128) - (a // 128)
cost = np.where(L >= 4, rows + 2, 0)
cs = np.cumsum(cost)
C_ = int(cs[-1])
G = 256
bounds = [0] + [int(np.searchsorted(cs, C_ // G * b + (C_ % G) * b // G, side="right")) for b in range(1, G)] + [R]
items = np.array([bounds[b + 1] - bounds[b] for b in range(G)])
rws = np.array([rows[bounds[b]:bounds[b + 1]].sum() for b in range(G)])
small = np.array([(rows[bounds[b]:bounds[b + 1]] <= 2).sum() for b in range(G)])
print("items per WG", q(items))
print("rows per WG", q(rws))
for name, x in (("items", items), ("rows", rws), ("small items", small), ("xcd", np.arange(G) % 8)):
    print(f"corr(end, {name}) = {np.corrcoef(wg_end, x)[0, 1]:+.3f}")
for x in range(8):
    print("xcd", x, "mean end %.1f" % wg_end[np.arange(G) % 8 == x].mean())
np.save(os.path.join(REPO, "gpurun_out", "wg_end.npy"), wg_end)
