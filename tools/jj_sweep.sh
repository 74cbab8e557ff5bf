#!/bin/bash
# Piece size x build at mid sizes (dev tool, round 6): the sorted path with
# each piece size forced, for the product build and an A/B build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 9
OUT=gpurun_out/${SESSION:-r06t}; mkdir -p "$OUT"
for rnd in 1 2; do
  for v in ${JJ_LIBS:-head nojj}; do
    lib=tools/ab/libconsus_crc32c_$v.so; [ "$v" = head ] && lib=consus_amd/lib/libconsus_crc32c.so
    for pl in ${JJ_PLOGS:-auto 12 13 14}; do
      envs=""; [ "$pl" != auto ] && envs="MI_CRC32C_SORT_PIECE_LOG2=$pl"
      env $envs timeout -k 10 120 python3 tools/mid_probe.py --lib "$lib" --path sorted --mib ${JJ_MIB:-64,128,256,512} --reps 200 > "$OUT/jj.out" 2>&1 || { cat "$OUT/jj.out"; exit 1; }
      grep -v "^path" "$OUT/jj.out" | sed "s/^/round $rnd $v p=$pl /"
    done
  done
done | tee "$OUT/jj_sweep.out"
