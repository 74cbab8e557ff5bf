#!/bin/bash
# Lane items before the team groups (MI_SORT_LANE_FIRST=1: every wave; 2: odd
# waves) against after them (the product), interleaved on one box: configs[2]
# (tools/ab.py --zipf) and the mid-size batches (mid_probe).  Dev tool, round 6;
# LF_LIBS names any variant builds (tools/build_variant.sh) to compare the same way.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 9
OUT=gpurun_out/${SESSION:-r06zj}; mkdir -p "$OUT"
LIBS="consus_amd/lib/libconsus_crc32c.so ${LF_LIBS:-tools/ab/libconsus_crc32c_lf1.so tools/ab/libconsus_crc32c_lf2.so}"
AB_ROUNDS=${AB_ROUNDS:-3} timeout -k 10 600 python3 -u tools/ab.py --zipf $LIBS > "$OUT/lane_first_zipf.out" 2>&1 || { tail -20 "$OUT/lane_first_zipf.out"; exit 1; }
cat "$OUT/lane_first_zipf.out"
for rnd in 1 2; do
  for lib in $LIBS; do
    echo "== round $rnd $lib"
    timeout -k 10 200 python3 -u tools/mid_probe.py --lib $lib --mib ${MID_MIB:-32,64,256,512} --reps 300 || exit 1
  done
done > "$OUT/lane_first_mid.out" 2>&1 || { tail -20 "$OUT/lane_first_mid.out"; exit 1; }
grep -v '^path=' "$OUT/lane_first_mid.out"
