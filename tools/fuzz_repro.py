"""Re-run one tests/test_gpu_fuzz.py round's batch through the sorted path and
the piece path and list the records where they differ (dev tool; the piece
path is the reference here, it matched the oracle in that round).

python tools/fuzz_repro.py ROUND GRID
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import consus_amd as E  # noqa: E402
from test_gpu_fuzz import random_lengths  # noqa: E402

rnd, grid = int(sys.argv[1]), sys.argv[2]
rng = np.random.default_rng(9000 + rnd)
count = int(rng.integers(1, 3000))
lengths = np.clip(random_lengths(rng, count), 0, None).astype(np.uint32)
layout = rng.integers(0, 3)
if layout == 0:
    offsets = np.zeros(count, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    offsets += np.uint64(rng.integers(0, 4096))
    size = int(offsets[-1] + lengths[-1]) + 64
else:
    size = int(lengths.max()) + int(rng.integers(1, 1 << 20))
    offsets = np.array([rng.integers(0, size - int(L) + 1) for L in lengths], dtype=np.uint64)
buf = rng.integers(0, 256, size, dtype=np.uint8)
inits = rng.integers(0, 2**32, count, dtype=np.uint32) if rng.integers(0, 2) else None
print("count", count, "layout", layout, "size", size, "inits", inits is not None,
      "max len", int(lengths.max()), "split records", int((lengths > 65536).sum()))
E.init(0)
data = E.DeviceBuffer(size)
data.upload(buf)
d_off, d_len, d_out = E.DeviceBuffer(count * 8), E.DeviceBuffer(count * 4), E.DeviceBuffer(count * 4)
d_off.upload(offsets)
d_len.upload(lengths)
d_ini = None
if inits is not None:
    d_ini = E.DeviceBuffer(count * 4)
    d_ini.upload(inits)
total = max(int(lengths.sum(dtype=np.uint64)), 1)
res = {}
for path in ("pieces", "sorted"):
    os.environ["MI_CRC32C_VARPATH"] = path
    if path == "sorted":
        os.environ["MI_CRC32C_SORTED_GRID"] = grid
    E.device_batch(data, d_off, d_len, count, d_out, inits=d_ini, total_bytes=total)
    res[path] = d_out.download(np.uint32, count)
bad = np.nonzero(res["pieces"] != res["sorted"])[0]
print("mismatches", bad.size)
for i in bad[:20]:
    print(f"rec {i} off {int(offsets[i])} (mod128 {int(offsets[i]) % 128}) len {int(lengths[i])} "
          f"pieces {int(res['pieces'][i]):#010x} sorted {int(res['sorted'][i]):#010x}")
