#!/bin/bash
# Stall breakdown of the sorted kernel by length class (dev tool): one
# rocprofv3 --pmc pass per workload (full configs[2]; only the records
# < 1 KiB; only those >= 1 KiB; the sorted path forced) with the SQ
# wait/active counters.
# WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES (quad-cycles).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/stall"
mkdir -p "$OUT"
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
for m in full keep drop; do
  envs="ZIPF_WARM=2 ZIPF_ROUNDS=1 MI_CRC32C_VARPATH=sorted"; [ "$m" = keep ] && envs="$envs ZIPF_KEEP_BELOW=1024"; [ "$m" = drop ] && envs="$envs ZIPF_DROP_BELOW=1024"
  (cd /tmp && env $envs timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$m" -o k -- python3 "$ROOT/tools/zipf_probe.py" > "$OUT/pmc_$m.log" 2>&1) || { tail -5 "$OUT/pmc_$m.log"; exit 1; }
  echo "== $m"; python3 "$ROOT/tools/pmc_summary.py" "$OUT/pmc_$m" crc32c_sorted_kernel
  rm -rf "$OUT/pmc_$m"
done | tee "$OUT/stall.out"
