"""bench.py's default N = 1 run on the CPU with full-size legs (tests/test_bench_line.py).

The engine is the CPU stand-in of tests/_bench_rank.py.  The legs that need
a GPU box (configs[2], configs[4], the PCIe-inclusive rate, the durable log,
the mid-size batches, the reference CPU baseline and the PMC pass) return
the records of a committed default line from a real session
(profiles/r05_bench_default_session_r05bs.json: per-run arrays, sample
strings, every key at its real size), so the line that main() assembles
and prints has the size and shape of the driver's.
"""
import copy
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import _bench_rank  # noqa: E402  (installs the consus_amd stand-in, imports bench)

bench = _bench_rank.bench
with open(os.path.join(HERE, "..", "profiles", "r05_bench_default_session_r05bs.json")) as f:
    FULL = json.loads(f.read().strip().splitlines()[-1])
LEG_OF = {"zipf": "config2_zipf", "stream": "config4_stream", "pcie4k": "config1_pcie_inclusive"}
# round 6: the durable-log leg has a third workload (storage faster than the
# front-end) of the same shape as the zipf one
FULL["durable_log"]["workloads"]["zipf_sink"] = copy.deepcopy(FULL["durable_log"]["workloads"]["zipf"])


def _leg(args, E, traffic=None):
    bench.progress(f"(stand-in) leg {args.config}")
    return copy.deepcopy(FULL[LEG_OF[args.config]])


bench.pmc_traffic = lambda args: (float(FULL["roofline"]["traffic"]), FULL["roofline"]["traffic_note"])
bench.run_secondary = _leg
bench.run_dlog = lambda args, compact=False: copy.deepcopy(FULL["durable_log"])
bench.run_mid = lambda E: copy.deepcopy(FULL["mid_batches"])
bench.cpu_baseline = lambda args: copy.deepcopy(FULL["cpu_baseline"])

if __name__ == "__main__":
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()
