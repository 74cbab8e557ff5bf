set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for L in base cx2 cx4; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/cx_$L" -o k --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/zipf_probe.py" "$GRAFT_REPO_ROOT/tools/ab/libconsus_crc32c_$L.so" > "$GRAFT_REPO_ROOT/gpurun_out/cx_$L.log" 2>&1) || { tail -5 gpurun_out/cx_$L.log; exit 1; }
  python3 - "$L" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/cx_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'sorted' in r['Name']:
        print(sys.argv[1], r['Name'][:32], r['Calls'], 'avg us', round(float(r['AverageNs']) / 1e3, 2), 'min us', round(float(r['MinNs']) / 1e3, 2))
PY
done
AB_ROUNDS=5 timeout -k 10 400 python tools/ab.py --zipf tools/ab/libconsus_crc32c_base.so tools/ab/libconsus_crc32c_cx2.so tools/ab/libconsus_crc32c_cx4.so
