"""Per-launch time of the headline kernel after the GPU has idled (dev tool).

bench.py's timed region is W = 5 warmup launches after the process starts,
then K = 20 timed ones, as the driver runs it.  This probe shows where those
launches sit on the device's clock ramp: it fills the 1M x 4 KiB batch, idles
IDLE seconds, then times LAUNCHES launches one at a time (HIP events on the
engine's stream, one sync per launch), and prints the per-launch times in
blocks plus the mean of launches 6-25 (bench.py's timed window at W = 5) and
of the last 100.

    python tools/ramp_probe.py [IDLE_S] [LAUNCHES]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import consus_amd as E  # noqa: E402

idle = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
n = int(sys.argv[2]) if len(sys.argv) > 2 else 600
R, L = 1 << 20, 4096
E.init(0)
data = E.DeviceBuffer(R * L)
out = E.DeviceBuffer(R * 4)
data.fill_splitmix64(0xC0DE)
E.sync()
time.sleep(idle)
t = []
for _ in range(n):
    E.timer_start()
    E.device_batch_fixed(data, L, L, R, out, asynchronous=True)
    t.append(E.timer_stop())
peak = 8000.0  # GB/s


def frac(ms):
    return R * L / (ms * 1e-3) / 1e9 / peak


for i in range(0, min(n, 100), 5):
    blk = t[i:i + 5]
    print(f"launches {i + 1:4d}-{i + len(blk):4d}: " + " ".join(f"{x:.4f}" for x in blk) +
          f"  mean {sum(blk) / len(blk):.4f} ms ({100 * frac(sum(blk) / len(blk)):.1f} %)")
w = t[5:25]
last = t[-100:]
print(f"bench window (launches 6-25): mean {sum(w) / len(w):.4f} ms ({100 * frac(sum(w) / len(w)):.1f} %)")
print(f"last 100: mean {sum(last) / len(last):.4f} ms ({100 * frac(sum(last) / len(last)):.1f} %)")
