#!/bin/bash
# rocprofv3 kernel trace of one bench.py config; prints per-kernel launch durations (us).
# usage: tools/prof_kernels.sh <tag> <bench args...>
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o k --output-format csv -- python3 "$ROOT/bench.py" "$@" > "$OUT/run.log" 2>&1 || { tail -20 "$OUT/run.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    d[r['Kernel_Name'].split('(')[0][-40:]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in d.items():
    v2 = sorted(v)
    print(f"{k:40s} n={len(v):3d} median={v2[len(v2)//2]:9.1f} us  min={v2[0]:9.1f}")
PY
