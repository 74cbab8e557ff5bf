"""A/B library builds (dev tool).

python tools/ab.py [--zipf] LIB_A.so LIB_B.so ...  -- each build is timed in
its own process, interleaved over three rounds, with tools/perf_probe.py
(1M x 4 KiB records) or tools/zipf_probe.py (config 3).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
args = sys.argv[1:]
zipf = "--zipf" in args
extra = [a for a in args if a.startswith("--") and a != "--zipf"]
libs = [a for a in args if not a.startswith("--")]
ablate = os.environ.get("AB_ALLOW_MISMATCH") == "1"  # ablation builds: wrong results expected
for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
    for lib in libs:
        cmd = [sys.executable, os.path.join(HERE, "zipf_probe.py"), lib] + extra if zipf else \
              [sys.executable, os.path.join(HERE, "perf_probe.py"), str(1 << 20), lib]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=180)
        line = (r.stdout.strip().splitlines() or ["<no output> " + r.stderr[-300:]])[-1]
        print(f"round {rnd} {os.path.basename(lib):28s} {line}", flush=True)
        # a GPU fault or a wrong digest ends the session: nothing more runs on the GPU
        if r.returncode != 0 or "HSA_STATUS_ERROR" in r.stdout + r.stderr or \
                ("MISMATCH" in line and not ablate):
            print(r.stderr[-2000:], file=sys.stderr)
            sys.exit(1)
