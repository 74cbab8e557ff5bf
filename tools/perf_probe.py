"""Quick device-resident throughput probe for the fixed kernel (dev tool).

The digest of the CRC vector is computed on the GPU (the oracle is test
infrastructure and is not imported outside tests/, smoke() and bench.py's
CPU-baseline leg); compare it with tests/golden/digests.json."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import consus_amd as E
if len(sys.argv) > 2:
    E.LIB_PATH = os.path.abspath(sys.argv[2])  # A/B builds (tools/ab.py)

count = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
L = 4096
E.init(0)
data = E.DeviceBuffer(count * L)
out = E.DeviceBuffer(count * 4)
data.fill_splitmix64(0xC0DE)
for _ in range(int(os.environ.get("PERF_WARM", "3"))):
    E.device_batch_fixed(data, L, L, count, out, asynchronous=True)
E.sync()
times = []
for _ in range(int(os.environ.get("PERF_N", "20"))):
    E.timer_start()
    E.device_batch_fixed(data, L, L, count, out, asynchronous=True)
    times.append(E.timer_stop())
crcs = out.download(np.uint32, count)
d = E.crc32c_device(out, count * 4)
x = int(np.bitwise_xor.reduce(crcs))
ms = float(np.median(times))
gb = count * L / 1e9
import json  # noqa: E402
gold = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                   "tests", "golden", "digests.json")))
want = gold["fixed_4096_seed0xc0de_per_1048576"]["block_digests"][0] if count == 1 << 20 else None
tag = "" if want is None else ("OK" if d == want else "MISMATCH")
print(f"count={count} median {ms:.4f} ms min {min(times):.4f} -> {gb/ms*1e3:.1f} GB/s "
      f"({count*L/2**30/ms*1e3:.1f} GiB/s)  digest {d:#010x} {tag} xor {x:#010x} first {crcs[0]:#010x}")
