#!/bin/bash
# Whole lane records hashed by the cost kernel (default) or as lane items of
# the hash kernel (MI_CRC32C_SORT_COST_LANES=0), interleaved on one box:
# configs[2] (zipf_probe) and the mid-size batches (mid_probe).  Dev tool, round 6.
# The knob belonged to the A/B build recorded in profiles/r06_lane_phase_ablation.txt
# (2); that form was not kept, so on the product both settings run the same code.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 9
OUT=gpurun_out/${SESSION:-r06zi}; mkdir -p "$OUT"
for rnd in 1 2 3; do
  for cl in 0 1; do
    r=$(MI_CRC32C_SORT_COST_LANES=$cl timeout -k 10 120 python3 tools/zipf_probe.py 2>&1 | tail -1) || { echo "$r"; exit 1; }
    echo "round $rnd cost_lanes=$cl $r"; case "$r" in *MISMATCH*) exit 1;; esac
  done
done | tee "$OUT/cost_lanes_zipf.out" || exit 1
for rnd in 1 2; do
  for cl in 0 1; do
    echo "== round $rnd cost_lanes=$cl"
    MI_CRC32C_SORT_COST_LANES=$cl timeout -k 10 200 python3 -u tools/mid_probe.py --mib ${MID_MIB:-32,64,128,256,512} --reps 300 || exit 1
  done
done > "$OUT/cost_lanes_mid.out" 2>&1 || { tail -20 "$OUT/cost_lanes_mid.out"; exit 1; }
tail -40 "$OUT/cost_lanes_mid.out"
