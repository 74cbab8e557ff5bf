"""A/B the fixed-length kernel across library builds (dev tool).

python tools/ab.py LIB_A.so LIB_B.so ...  -- each build is timed in its own
process, interleaved over three rounds, with tools/perf_probe.py.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
libs = sys.argv[1:]
for rnd in range(3):
    for lib in libs:
        r = subprocess.run([sys.executable, os.path.join(HERE, "perf_probe.py"), str(1 << 20), lib],
                           capture_output=True, text=True, timeout=120)
        line = (r.stdout.strip().splitlines() or ["<no output> " + r.stderr[-300:]])[-1]
        print(f"round {rnd} {os.path.basename(lib):28s} {line}", flush=True)
