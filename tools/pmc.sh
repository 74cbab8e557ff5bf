#!/bin/bash
# PMC counters per kernel for one bench.py config (one rocprofv3 --pmc pass per
# counter set; no tracing domains).  Prints the median per kernel.
# usage: tools/pmc.sh <tag> "<counters>" <bench args...>
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
CTRS="$1"; shift
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT" -o k -- python3 "$ROOT/bench.py" "$@" > "$OUT/run.log" 2>&1 || { tail -20 "$OUT/run.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    d[r['Kernel_Name'].split('(')[0][-34:]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in d.items():
    print(k, "  ".join(f"{c}={sorted(v)[len(v)//2]:.4g}" for c, v in sorted(cs.items())))
PY
