#!/bin/bash
# Sorted-kernel stamps at one mid size for several stamp builds and pieces (dev tool, round 6).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 9
OUT=gpurun_out/${SESSION:-r06z}; mkdir -p "$OUT"
for v in ${ABL_LIBS:-stamp stampabl1 stampabl2}; do
  for pl in ${ABL_PLOGS:-13 14}; do
    echo "== $v piece 2^$pl ${ABL_MIB:-256} MiB"
    MI_CRC32C_SORT_PIECE_LOG2=$pl timeout -k 10 120 python3 tools/sort_stamps.py tools/ab/libconsus_crc32c_$v.so --mib ${ABL_MIB:-256} | grep -v "^  e\|^  b\|^  r\|^records" || exit 1
  done
done | tee "$OUT/stamp_abl.out"
