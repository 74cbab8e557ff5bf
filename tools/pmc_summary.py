"""Median per kernel of every counter in a rocprofv3 --pmc csv directory (dev tool).

python tools/pmc_summary.py DIR [KERNEL_SUBSTRING ...]
"""
import collections
import csv
import glob
import sys

d = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"].split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
want = sys.argv[2:]
for k, cs in sorted(d.items()):
    if want and not any(w in k for w in want):
        continue
    n = max(len(v) for v in cs.values())
    print(f"{k} (n={n})  " + "  ".join(f"{c}={sorted(v)[len(v) // 2]:.4g}" for c, v in sorted(cs.items())))
