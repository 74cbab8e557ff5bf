#!/bin/bash
# rocprofv3 kernel trace of tools/zipf_probe.py for one library build (dev tool):
#   tools/prof_probe.sh TAG LIB.so   -> per-kernel median durations
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; LIB="$2"
OUT="$ROOT/gpurun_out/pp_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
LIB="$(cd "$ROOT" && realpath "$LIB")"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT" -o k --output-format csv -- python3 "$ROOT/tools/zipf_probe.py" "$LIB" > "$OUT/run.log" 2>&1 || { tail -20 "$OUT/run.log"; exit 1; }
tail -1 "$OUT/run.log"
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
