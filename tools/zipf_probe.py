"""Config-3 (Zipf) step time for one library build (dev tool, tools/ab.py).

python tools/zipf_probe.py [LIB.so]  -- 100 warm-up steps, then 5 rounds of 50
back-to-back steps timed with HIP events; prints the median and minimum
per-step time of the rounds and checks the digest against the golden one.
"""
import json
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
R = 1 << 20
off, ln, total = W.zipf_records(R)
# ZIPF_DROP_BELOW=n / ZIPF_KEEP_BELOW=n: zero the lengths of the records
# shorter / not shorter than n bytes (cost of one length class; wrong digest)
if os.environ.get("ZIPF_DROP_BELOW"):
    ln = np.where(ln < int(os.environ["ZIPF_DROP_BELOW"]), 0, ln).astype(ln.dtype)
if os.environ.get("ZIPF_KEEP_BELOW"):
    ln = np.where(ln < int(os.environ["ZIPF_KEEP_BELOW"]), ln, 0).astype(ln.dtype)
# ZIPF_ALIGN=n: every record starts on an n-byte boundary (gaps between them;
# no 128-B line shared by two records at n = 128; wrong digest by design)
if int(os.environ.get("ZIPF_ALIGN", "0") or 0) > 0:
    al = int(os.environ["ZIPF_ALIGN"])
    padded = ((ln.astype(np.uint64) + np.uint64(al - 1)) // np.uint64(al)) * np.uint64(al)
    off = np.zeros(R, dtype=np.uint64)
    off[1:] = np.cumsum(padded[:-1], dtype=np.uint64)
    total = int(off[-1] + padded[-1])
data = E.DeviceBuffer(total + 16)
data.fill_splitmix64(W.DATA_SEED)
d_off, d_len, out = E.DeviceBuffer(R * 8), E.DeviceBuffer(R * 4), E.DeviceBuffer(R * 4)
d_off.upload(off)
d_len.upload(ln)
hint = int(ln.sum(dtype=np.uint64))
WARM, ROUNDS = int(os.environ.get("ZIPF_WARM", "100")), int(os.environ.get("ZIPF_ROUNDS", "5"))
for _ in range(WARM):
    E.device_batch(data, d_off, d_len, R, out, total_bytes=hint, asynchronous=True)
E.sync()
rounds = []
for _ in range(ROUNDS):
    E.timer_start()
    for _ in range(50):
        E.device_batch(data, d_off, d_len, R, out, total_bytes=hint, asynchronous=True)
    rounds.append(E.timer_stop() / 50)
dig = E.crc32c_device(out, R * 4)
with open(os.path.join(REPO, "tests", "golden", "digests.json")) as f:
    gold = json.load(f)["zipf_seed0x5eed_data0xda7a5eed_1048576"]["digest"]
ms = float(np.median(rounds))
print(f"zipf {hint} B median {ms:.4f} ms min {min(rounds):.4f} -> {total / ms / 1e6:.1f} GB/s "
      f"({100 * total / ms / 1e6 / 8000:.1f} %) digest {dig:#010x} {'OK' if dig == gold else 'MISMATCH'}")
