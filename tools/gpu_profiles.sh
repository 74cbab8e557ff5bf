#!/bin/bash
# Regenerate the committed evidence under profiles/ (one GPU session):
# parity tests, smoke, every bench config, rocprofv3 --kernel-trace --stats
# summaries of the device-resident configs, and a 2-rank rehearsal of the
# N > 1 path on the one GPU.  Every GPU step has its own time limit and the
# script stops at the first failure.  Output: gpurun_out/prof_<TAG>/.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03}"
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT" || exit 9
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "FAILED $name"; tail -20 "$OUT/$name.err"; exit 1; }
  tail -2 "$OUT/$name.out"
}
stats() {  # config extra-args...
  local c=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_$c" -o k --output-format csv \
     -- python3 "$ROOT/bench.py" --config "$c" --no-cpu --no-pmc --no-legs --sustain-seconds 0 --steps 30 --warmup 300 "$@" > "$OUT/rocprof_$c.log" 2>&1) \
     || { echo "FAILED rocprof $c"; tail -20 "$OUT/rocprof_$c.log"; exit 1; }
  cp "$(find "$OUT/rocprof_$c" -name '*kernel_stats.csv' | head -1)" "$OUT/${c}_kernel_stats.csv"
}
if [ "$2" = "stats" ]; then  # only the rocprof legs: tools/gpu_profiles.sh TAG stats CONFIG...
  shift 2; for c in "$@"; do stats "$c"; done; echo "ALL OK"; exit 0
fi
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_fixed4k 600 python bench.py
run bench_zipf 600 python bench.py --config zipf --no-cpu
run bench_single 300 python bench.py --config single --no-cpu
run bench_stream 300 python bench.py --config stream --no-cpu
run bench_pcie4k 300 python bench.py --config pcie4k --no-cpu
run bench_dlog 300 python bench.py --config dlog --steps 30
run shard_overhead 300 python tools/shard_probe.py
stats fixed4k
stats zipf
stats single
run bench_n2_rehearsal 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --share-device --steps 5 --warmup 2 --no-cpu
run bench_single_split_n2_rehearsal 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config single --share-device --steps 10 --warmup 2
run bench_zipf_n2_rehearsal 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --config zipf --share-device --steps 10 --warmup 2
echo "ALL OK"
