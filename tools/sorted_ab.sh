#!/bin/bash
# sorted-path session (dev tool): parity tests, then A/B of library builds on configs[2]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 9
OUT=gpurun_out/sorted; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sorted.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_sorted.log 2>&1 || { tail -40 $OUT/pytest_sorted.log; exit 1; }
tail -1 $OUT/pytest_sorted.log
AB_ALLOW_MISMATCH=1 AB_ROUNDS=${AB_ROUNDS:-2} timeout -k 10 500 python tools/ab.py --zipf "$@"
