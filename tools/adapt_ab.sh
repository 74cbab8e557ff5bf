#!/bin/bash
# Adaptive per-XCD shares on/off, interleaved on one box (dev tool, round 6).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 9
OUT=gpurun_out/${SESSION:-r06zd}; mkdir -p "$OUT"
for rnd in 1 2 3 4; do
  for a in 0 1; do
    r=$(MI_CRC32C_SORT_ADAPT=$a timeout -k 10 120 python3 tools/zipf_probe.py 2>&1 | tail -1) || { echo "$r"; exit 1; }
    echo "round $rnd adapt=$a $r"; case "$r" in *MISMATCH*) exit 1;; esac
  done
done | tee "$OUT/adapt_ab.out"
for rnd in 1 2; do
  for a in 0 1; do
    MI_CRC32C_SORT_ADAPT=$a timeout -k 10 120 python3 tools/mid_probe.py --path sorted --mib ${AMIB:-64,128,256,512,1024} --reps 200 > "$OUT/am.out" 2>&1 || { cat "$OUT/am.out"; exit 1; }
    grep -v "^path" "$OUT/am.out" | sed "s/^/round $rnd adapt=$a /"
  done
done | tee -a "$OUT/adapt_ab.out"
for a in 0 1; do
  echo "== stamps adapt=$a"
  MI_CRC32C_SORT_ADAPT=$a timeout -k 10 120 python3 tools/sort_stamps.py tools/ab/libconsus_crc32c_stamp.so | grep -v "^  [ebr]" || exit 1
done | tee -a "$OUT/adapt_ab.out"
