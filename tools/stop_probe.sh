#!/bin/bash
# Prologue phases of the sorted kernel (dev tool): kernel time of the
# MI_SORT_STOP builds (results wrong by design) under rocprofv3 --stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 9
export TMPDIR=/tmp
for L in "$@"; do
  t=$(basename "$L" .so)
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/stop_$t" -o k --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/zipf_probe.py" "$GRAFT_REPO_ROOT/$L" > "$GRAFT_REPO_ROOT/gpurun_out/stop_$t.log" 2>&1) || { tail -5 "gpurun_out/stop_$t.log"; exit 1; }
  python3 - "$t" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/stop_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'sorted' in r['Name']:
        print(f"{sys.argv[1]:34s} {r['Name'][8:30]:22s} calls {r['Calls']} avg {float(r['AverageNs']) / 1e3:8.2f} us min {float(r['MinNs']) / 1e3:8.2f} us")
PY
done
