#!/bin/bash
# Ring depth x piece size at mid sizes through one A/B build (dev tool, round 6).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 9
OUT=gpurun_out/${SESSION:-r06v}; mkdir -p "$OUT"
lib=tools/ab/libconsus_crc32c_${RING_LIB:-ring8}.so
for rnd in 1 2; do
  for rg in ${RINGS:-4 8}; do
    for pl in ${PLOGS:-auto 12 13}; do
      envs="MI_CRC32C_SORT_RING=$rg"; [ "$pl" != auto ] && envs="$envs MI_CRC32C_SORT_PIECE_LOG2=$pl"
      env $envs timeout -k 10 120 python3 tools/mid_probe.py --lib "$lib" --path sorted --mib ${RMIB:-16,64,128,256,512} --reps 200 > "$OUT/rs.out" 2>&1 || { cat "$OUT/rs.out"; exit 1; }
      grep -v "^path" "$OUT/rs.out" | sed "s/^/round $rnd ring=$rg p=$pl /"
    done
  done
done | tee "$OUT/ring_sweep.out"
