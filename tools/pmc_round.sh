#!/bin/bash
# SQ counters of the headline and configs[2] steps (one --pmc pass each) ->
# gpurun_out/pmc_sq.txt, the format of profiles/rNN_pmc_sq_counters.txt (dev tool)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
O="$ROOT/gpurun_out/pmc_sq.txt"
echo "# tools/pmc.sh: rocprofv3 --pmc $C" > "$O"
echo "# (one pass per config, no tracing domains; median over the run's dispatches of each kernel)" >> "$O"
for c in fixed4k zipf; do
  echo "# $c: bench.py --config $c --no-cpu --no-pmc --sustain-seconds 0 --steps 3 --warmup 1" >> "$O"
  bash "$ROOT/tools/pmc.sh" "sq_$c" "$C" --config $c --no-cpu --no-pmc --sustain-seconds 0 --steps 3 --warmup 1 >> "$O" || exit 1
  echo >> "$O"
done
cat "$O"
