"""Per-kernel median durations and the median idle gap before each kernel in a
rocprofv3 kernel trace (dev tool): where a multi-launch batch spends time.

python tools/kernel_gaps.py k_kernel_trace.csv [last_n]
"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
rows = rows[-last:]
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
prev_end = None
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("mi_crc::", "")[:48]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[name].append((e - s) / 1e3)
    if prev_end is not None:
        gap[name].append((s - prev_end) / 1e3)
    prev_end = e
print(f"{'kernel':48s} {'n':>6s} {'median us':>10s} {'gap before us':>14s}")
for k in dur:
    g = statistics.median(gap[k]) if gap[k] else float("nan")
    print(f"{k:48s} {len(dur[k]):6d} {statistics.median(dur[k]):10.2f} {g:14.2f}")
