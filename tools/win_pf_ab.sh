#!/bin/bash
# Window kernel: table sets read into L2 beside the rows (MI_WIN_PF=1) against
# the product, interleaved on one box, configs[2] records cut to N MiB on the
# window path (tools/mid_probe.py).  Dev tool, round 6.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 9
OUT=gpurun_out/${SESSION:-r06zk}; mkdir -p "$OUT"
for rnd in 1 2 3; do
  for lib in consus_amd/lib/libconsus_crc32c.so ${PF_LIBS:-tools/ab/libconsus_crc32c_winpf.so}; do
    echo "== round $rnd $lib"
    timeout -k 10 200 python3 -u tools/mid_probe.py --path window --lib $lib --mib ${MID_MIB:-1,4,8,16,20} --reps 300 || exit 1
  done
done > "$OUT/win_pf.out" 2>&1 || { tail -20 "$OUT/win_pf.out"; exit 1; }
grep -v '^path=' "$OUT/win_pf.out"
