"""Debug a sorted-path batch with help on (dev tool): the random-lengths case of
tests/test_gpu_sorted.py (seed 1) with 64 KiB pieces; prints the mismatching
records under several help settings."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

import ctypes as C  # noqa: E402

import consus_amd as E  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

if len(sys.argv) > 1:
    E.LIB_PATH = os.path.abspath(sys.argv[1])
E.init(0)
O = Oracle()
rng = np.random.default_rng(101)
count = 40_000
lengths = rng.integers(0, 20_000, count).astype(np.uint32)
lengths[rng.integers(0, count, 2000)] = rng.integers(0, 5, 2000)
offsets = np.zeros(count, dtype=np.uint64)
steps = lengths[:-1].astype(np.uint64) + rng.integers(0, 10, count - 1).astype(np.uint64)
offsets[1:] = np.cumsum(steps)
offsets += np.uint64(int(rng.integers(0, 128)))
end = int(offsets[-1]) + int(lengths[-1])
buf = rng.integers(0, 256, end + 64, dtype=np.uint8)
want = O.batch(buf, offsets, lengths)
data = E.DeviceBuffer(buf.size)
data.upload(buf)
d_off, d_len, d_out = E.DeviceBuffer(count * 8), E.DeviceBuffer(count * 4), E.DeviceBuffer(count * 4)
d_off.upload(offsets)
d_len.upload(lengths)
os.environ["MI_CRC32C_VARPATH"] = "sorted"
os.environ["MI_CRC32C_SORT_PIECE_LOG2"] = "16"
for cfg in [("0", "0", "0"), ("1", "0", "1"), ("1", "0", str(1 + 16 * 9)), ("1", "0", str(1 + 16 * 1)),
            ("1", "0", str(1 + 16 * 8)), ("1", "0", "0")]:
    os.environ["MI_CRC32C_SORT_HELP"], os.environ["MI_CRC32C_SORT_HELP_DELAY_US"], \
        os.environ["MI_CRC32C_SORT_HELP_DBG"] = cfg
    d_out.upload(np.zeros(count, dtype=np.uint32))
    E.device_batch(data, d_off, d_len, count, d_out, total_bytes=int(lengths.sum(dtype=np.uint64)))
    got = d_out.download(np.uint32, count)
    bad = np.nonzero(got != want)[0]
    print(f"help={cfg[0]} delay={cfg[1]} dbg={cfg[2]}: {bad.size} bad; first {bad[:12].tolist()} "
          f"lengths {lengths[bad[:12]].tolist()}", flush=True)
    if len(sys.argv) > 1:
        L = E.lib()
        L.mi_debug_sort_dbg.argtypes = [C.c_void_p, C.c_size_t]
        dbg = np.zeros(8200, dtype=np.uint32)
        assert L.mi_debug_sort_dbg(dbg.ctypes.data, dbg.size) == 0
        print("  wg0 s0 res_end res_final n_groups lane_base helpable", dbg[8192:8198].tolist())
        print("  wg0 W[0:160]", " ".join(f"{x:08x}" for x in dbg[:160]), flush=True)
