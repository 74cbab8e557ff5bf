#!/bin/bash
# configs[2] with the 2- and 4-row rings interleaved on one box (dev tool, round 6).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 9
OUT=gpurun_out/${SESSION:-r06zg}; mkdir -p "$OUT"
for rnd in 1 2 3; do
  for rg in 2 4; do
    r=$(MI_CRC32C_SORT_RING=$rg timeout -k 10 120 python3 tools/zipf_probe.py 2>&1 | tail -1) || { echo "$r"; exit 1; }
    echo "round $rnd ring=$rg $r"; case "$r" in *MISMATCH*) exit 1;; esac
  done
done | tee "$OUT/ring_zipf_ab.out"
