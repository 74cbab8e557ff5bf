set -o pipefail
for r in 1 2; do
 for v in "" "ZIPF_DROP_BELOW=1024" "ZIPF_KEEP_BELOW=1024" "ZIPF_DROP_BELOW=256" "ZIPF_KEEP_BELOW=256"; do
  echo -n "[$v] "; env $v timeout -k 10 120 python tools/zipf_probe.py | tail -1
 done
done
