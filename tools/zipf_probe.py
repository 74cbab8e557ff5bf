"""Config-3 (Zipf) step time for one library build (dev tool).

python tools/zipf_probe.py [LIB.so]  -- prints median/min event time and the digest.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import consus_amd as E  # noqa: E402
args = [a for a in sys.argv[1:] if not a.startswith("--")]
PACKED = "--packed" in sys.argv  # MI_CRC32C_PACKED: the stream path
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
# ZIPF_PACK=1: the same records moved back to back (address locality test)
if os.environ.get("ZIPF_PACK"):
    off = np.concatenate([[0], np.cumsum(ln[:-1].astype(np.uint64))]).astype(off.dtype) + off[0]
data = E.DeviceBuffer(total + 16)
data.fill_splitmix64(W.DATA_SEED)
d_off, d_len, out = E.DeviceBuffer(R * 8), E.DeviceBuffer(R * 4), E.DeviceBuffer(R * 4)
d_off.upload(off)
d_len.upload(ln)
for _ in range(3):
    E.device_batch(data, d_off, d_len, R, out, total_bytes=total, packed=PACKED)
E.sync()
times = []
for _ in range(15):
    E.timer_start()
    E.device_batch(data, d_off, d_len, R, out, total_bytes=total, asynchronous=True,
                   packed=PACKED)
    times.append(E.timer_stop())
dig = E.crc32c_device(out, R * 4)
with open(os.path.join(REPO, "tests", "golden", "digests.json")) as f:
    gold = json.load(f)["zipf_seed0x5eed_data0xda7a5eed_1048576"]["digest"]
ms = float(np.median(times))
print(f"{'stream' if PACKED else 'var'} zipf {int(ln.sum(dtype=np.uint64))} B median {ms:.4f} ms min {min(times):.4f} -> {total / ms / 1e6:.1f} GB/s "
      f"digest {dig:#010x} {'OK' if dig == gold else 'MISMATCH'}")
