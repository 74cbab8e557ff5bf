#!/bin/bash
# Which kind of box is this (dev tool, round 6): its clocks, then configs[2]
# and the headline timed, then the sorted kernel's stamps on configs[2].
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 9
OUT=gpurun_out/${SESSION:-r06zc}; mkdir -p "$OUT"
{
  echo "== clocks"; (timeout 30 rocm-smi --showclocks 2>&1 || true) | grep -v "^$" | head -40
  echo "== configs[2]"; timeout -k 10 120 python3 tools/zipf_probe.py | tail -1 || exit 1
  echo "== headline"; timeout -k 10 120 python3 tools/perf_probe.py $((1 << 20)) | tail -1 || exit 1
  echo "== stamps"; timeout -k 10 120 python3 tools/sort_stamps.py tools/ab/libconsus_crc32c_stamp.so || exit 1
} 2>&1 | tee "$OUT/box_probe.out"
