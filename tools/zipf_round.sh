set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prof_r02z; mkdir -p $OUT
timeout -k 10 300 python bench.py --config zipf --no-cpu > $OUT/bench_zipf.out 2> $OUT/bench_zipf.err || exit 1
cat $OUT/bench_zipf.out
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/rocprof_zipf -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config zipf --no-cpu --no-pmc --steps 30 --warmup 5 > $GRAFT_REPO_ROOT/$OUT/rocprof_zipf.log 2>&1 || exit 2
echo done
