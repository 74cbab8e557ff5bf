#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT" || exit 9
STEPS="${STEPS:-tests smoke bench prof}"
for s in $STEPS; do
  case "$s" in
    tests) timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
           tail -3 "$OUT/pytest_gpu.log" ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 2; }
           tail -1 "$OUT/smoke.log" ;;
    bench) timeout -k 10 600 python bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 3; }
           cat "$OUT/bench.json" ;;
    prof)  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --no-pmc > "$OUT/prof.log" 2>&1) || { tail -20 "$OUT/prof.log"; exit 4; }
           find "$OUT/prof" -name "*kernel_stats.csv" -exec head -12 {} \; ;;
    *) python "$s" || exit 5 ;;
  esac
done
