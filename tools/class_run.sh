#!/bin/bash
# PMC counters of the sorted kernel on one length class (dev tool)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
for v in ${CLASSES:-256 0}; do
  O="$ROOT/gpurun_out/cls_$v$(basename "${ZIPF_LIB:-}" .so)"; mkdir -p "$O"
  if [ $v = 0 ]; then E=""; else E="ZIPF_KEEP_BELOW=$v"; fi
  env $E timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$O" -o k -- python3 "$ROOT/tools/zipf_probe.py" $ZIPF_LIB > "$O/run.log" 2>&1 || { tail -5 "$O/run.log"; exit 1; }
  python3 - "$O" "$v" "${ZIPF_LIB:-default}" <<'PY'
import csv, glob, sys, collections, os
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'crc32c_sorted_kernel' in r['Kernel_Name']:
        d[r['Counter_Name']].append(float(r['Counter_Value']))
print("keep_below", sys.argv[2], os.path.basename(sys.argv[3]), "  ".join(f"{c}={sorted(v)[len(v)//2]:.4g}" for c, v in sorted(d.items())))
PY
done
