#!/bin/bash
# LDS bank-conflict share of the headline kernel for A/B library builds (dev
# tool): one rocprofv3 --pmc pass per build over tools/perf_probe.py.
# usage: tools/lds_conflicts.sh LIB.so ...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename "$lib" .so)
  OUT="$ROOT/gpurun_out/ldsc_$tag"; mkdir -p "$OUT"
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d "$OUT" -o k -- python3 "$ROOT/tools/perf_probe.py" 1048576 "$ROOT/$lib" > "$OUT/run.log" 2>&1 || { tail -20 "$OUT/run.log"; exit 1; }
  python3 - "$OUT" "$tag" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if 'fixed_pipe' in r['Kernel_Name']:
        d['k'][r['Counter_Name']].append(float(r['Counter_Value']))
m = {c: sorted(v)[len(v) // 2] for c, v in d['k'].items()}
print(f"{sys.argv[2]:28s} conflict {m['SQ_LDS_BANK_CONFLICT']:.4g} active {m['SQ_LDS_IDX_ACTIVE']:.4g} "
      f"-> {100 * m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.2f} %  lds insts {m['SQ_INSTS_LDS']:.4g}")
PY
done
