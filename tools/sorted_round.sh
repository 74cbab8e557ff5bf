#!/bin/bash
# GPU session for the sorted variable-length path: its parity tests, the
# configs[2] golden tests, then the configs[2] bench line (dev tool).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 9
OUT=gpurun_out/sorted; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sorted.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_sorted.log 2>&1 || { tail -40 $OUT/pytest_sorted.log; exit 1; }
tail -2 $OUT/pytest_sorted.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "zipf or config2 or config3 or var_" > $OUT/pytest_zipf.log 2>&1 || { tail -40 $OUT/pytest_zipf.log; exit 2; }
tail -2 $OUT/pytest_zipf.log
timeout -k 10 300 python bench.py --config zipf --no-cpu > $OUT/bench_zipf.json 2> $OUT/bench_zipf.err || { tail -20 $OUT/bench_zipf.err; exit 3; }
cat $OUT/bench_zipf.json
