#!/bin/bash
# GPU session (dev tool): the GPU suite, then the measurement probes
# named on the command line.  Every GPU step has its own limit; the script
# stops at the first failure.  Output: gpurun_out/$SESSION/<step>.* (SESSION default r04)
#   tools/session.sh tests route crossover rehearsal dlog zipf fixed ...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${SESSION:-r06}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT" || exit 9
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "FAILED $name rc=$?"; tail -n 30 "$OUT/$name.out" "$OUT/$name.err"; exit 1; }
  tail -3 "$OUT/$name.out"
}
while [ $# -gt 0 ]; do
  step=$1; shift
  case $step in
    tests) run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    window) run pytest_window 300 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_errors.py -x -q --timeout 120 --timeout-method thread &&
            for rnd in 1 2; do for pth in window sorted; do
              run mid_${pth}_$rnd 200 python3 tools/mid_probe.py --path $pth --mib ${WIN_MIB:-1,2,4,8,16} --reps 300
            done; done ;;
    winblock) for rnd in 1 2; do for b in 64 256; do
             MI_CRC32C_WIN_BLOCK=$b timeout -k 10 120 python3 tools/mid_probe.py --path window --mib ${WIN_MIB:-1,2,4,8,16} --reps 300 > "$OUT/w.out" 2>&1 || { cat "$OUT/w.out"; exit 1; }; grep -v "^path" "$OUT/w.out" | sed "s/^/round $rnd block=$b /"
           done; done | tee "$OUT/winblock.out" ;;
    fetchsplit) C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
             for cfg in fixed4k zipf; do
               (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/fs_$cfg" -o k -- python3 "$ROOT/bench.py" --child-pmc --config $cfg --records-per-rank 1048576 --record-bytes 4096 > "$OUT/fs_$cfg.log" 2>&1) || { tail -5 "$OUT/fs_$cfg.log"; exit 1; }
               echo "== $cfg"; python3 tools/pmc_summary.py "$OUT/fs_$cfg" crc32c_fixed_pipe crc32c_sorted_kernel sorted_cost_kernel
             done | tee "$OUT/fetchsplit.out"
             for m in keep drop; do
               envs="ZIPF_WARM=2 ZIPF_ROUNDS=1 MI_CRC32C_SORT_PIECE_LOG2=16 MI_CRC32C_SORT_RING=2"; [ "$m" = keep ] && envs="$envs ZIPF_KEEP_BELOW=1024"; [ "$m" = drop ] && envs="$envs ZIPF_DROP_BELOW=1024"
               (cd /tmp && env $envs timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/fs_$m" -o k -- python3 "$ROOT/tools/zipf_probe.py" > "$OUT/fs_$m.log" 2>&1) || { tail -5 "$OUT/fs_$m.log"; exit 1; }
               echo "== $m"; python3 tools/pmc_summary.py "$OUT/fs_$m" crc32c_sorted_kernel sorted_cost_kernel
             done | tee -a "$OUT/fetchsplit.out"
             rm -rf "$OUT"/fs_*/ ;;
    stealab) for rnd in 1 2 3; do for cfg in ${STEAL_CFGS:-r05d_0 head_0 head_4 head_8 head_16}; do
               set -- ${cfg/_/ }; lib=tools/ab/libconsus_crc32c_$1.so; [ "$1" = head ] && lib=consus_amd/lib/libconsus_crc32c.so
               echo -n "round $rnd lib=$1 steal=$2 "; MI_CRC32C_SORT_STEAL=$2 timeout -k 10 120 python3 tools/zipf_probe.py $lib > "$OUT/z.out" 2>&1 || { cat "$OUT/z.out"; exit 1; }; tail -1 "$OUT/z.out"
             done; done | tee "$OUT/stealab.out"
             for v in ${STEAL_MID:-0 4 8}; do MI_CRC32C_SORT_STEAL=$v timeout -k 10 120 python3 tools/mid_probe.py --path sorted --mib 64,256 --reps 200 ${MID_LIB:+--lib $MID_LIB} > "$OUT/w.out" 2>&1 || { cat "$OUT/w.out"; exit 1; }; grep -v "^path" "$OUT/w.out" | sed "s/^/steal=$v /"; done | tee -a "$OUT/stealab.out" ;;
    midab) for rnd in 1 2 3; do for v in ${MIDAB_LIBS:-pre768 head}; do
             lib=tools/ab/libconsus_crc32c_$v.so; [ "$v" = head ] && lib=consus_amd/lib/libconsus_crc32c.so
             timeout -k 10 120 python3 tools/mid_probe.py --lib $lib --mib ${MID_MIB:-1,2,4,8,12,16,20,24,28} --reps 300 > "$OUT/w.out" 2>&1 || { cat "$OUT/w.out"; exit 1; }; grep -v "^path" "$OUT/w.out" | sed "s/^/round $rnd $v /"
           done; done | tee "$OUT/midab.out" ;;
    midhead) run mid_head 300 python3 -u tools/mid_probe.py --mib ${MID_MIB:-1,2,4,8,16,32,64,256} --reps 300 ;;
    winbig) for rnd in 1 2; do for cfg in ${WINBIG_CFGS:-"window_8_256" "window_16_256" "window_8_64" "sorted_0_0"}; do
             set -- ${cfg//_/ }; MI_CRC32C_WIN_PIPE=${4:-0} MI_CRC32C_WIN_MAX_COUNT=16384 MI_CRC32C_WIN_ROWS=$2 MI_CRC32C_WIN_BLOCK=$3 timeout -k 10 120 python3 tools/mid_probe.py --path $1 --mib ${WIN_MIB:-16,32,48,64} --reps 200 > "$OUT/w.out" 2>&1 || { cat "$OUT/w.out"; exit 1; }; grep -v "^path" "$OUT/w.out" | sed "s/^/round $rnd rows=$2 block=$3 pipe=${4:-0} /"
           done; done | tee "$OUT/winbig.out" ;;
    winrows) for rnd in 1 2; do for r in ${WIN_ROWS:-4 8 16}; do
             MI_CRC32C_WIN_ROWS=$r timeout -k 10 120 python3 tools/mid_probe.py --path window --mib ${WIN_MIB:-1,2,4} --reps 300 > "$OUT/w.out" 2>&1 || { cat "$OUT/w.out"; exit 1; }; grep -v "^path" "$OUT/w.out" | sed "s/^/round $rnd rows=$r /"
           done; done | tee "$OUT/winrows.out" ;;
    wskip) for rnd in 1 2; do for v in ${WSKIP_LIBS:-w0 wskip1 wskip2 wskip4 wskip3 wskip7}; do
             timeout -k 10 120 python3 tools/mid_probe.py --lib tools/ab/libconsus_crc32c_$v.so --path window --mib ${WIN_MIB:-1,4,16} --reps 300 > "$OUT/w.out" 2>&1 || { cat "$OUT/w.out"; exit 1; }; grep -v "^path" "$OUT/w.out" | sed "s/^/round $rnd /"
           done; done | tee "$OUT/wskip.out" ;;
    errtests) run pytest_err 600 python -u -m pytest tests/test_gpu_errors.py tests/test_gpu_window.py -x -q --timeout 300 --timeout-method thread ;;
    wghw) run wg_hw 300 python3 tools/wg_hw_probe.py tools/ab/libconsus_crc32c_stamp.so "$OUT/wg_hw.npz" --launches ${WGHW_LAUNCHES:-12} ;;
    dlogtl) for rnd in 1 2 3; do for eng in ${DLOGTL_ENGINES:-gpu fake_pinned fake refscheme}; do
              envs="DLOG_ENTRY=zipf DLOG_TIMELINE=$OUT/tl_${eng}_$rnd.txt"
              case $eng in fake_pinned) envs="$envs FAKE_CRC=1 DLOG_PINNED=1";; fake) envs="$envs FAKE_CRC=1";;
                refscheme) envs="$envs REF_CRC_SO=$ROOT/oracle/_ref/libref_crc32c.so REF_SCHEME=1";; gpu_unpinned) envs="$envs DLOG_PINNED=0";; esac
              rm -rf /dev/shm/dltl; env $envs timeout -k 10 120 ./tools/dlog_bench /dev/shm/dltl 8 ${DLOGTL_PER:-25000} 0 0 > "$OUT/dl.out" 2> "$OUT/dl.err" || { cat "$OUT/dl.err"; rm -rf /dev/shm/dltl; exit 1; }
              echo "round $rnd $eng $(cat "$OUT/dl.out")"
            done; done > "$OUT/dlogtl.out"; rm -rf /dev/shm/dltl; cut -c1-200 "$OUT/dlogtl.out" ;;
    sortedtests) run pytest_sorted 900 python -u -m pytest tests/test_gpu_sorted.py tests/test_gpu_fuzz.py tests/test_gpu_errors.py -x -q --timeout 300 --timeout-method thread ;;
    soak) FUZZ_ROUNDS=${SOAK_ROUNDS:-1000} run fuzz_soak 900 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    route) run route_probe 300 ./tools/route_probe 200 ;;
    flush) run flush_probe 300 ./tools/flush_probe 1000 ;;
    launch) run launch_probe 120 ./tools/launch_probe 2000 && run launch_probe_spin 120 ./tools/launch_probe 2000 spin ;;
    crossover) run crossover 400 python3 -u tools/varpath_crossover.py ;;
    varprof) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/varprof" -o k -- python3 "$ROOT/tools/varpath_crossover.py" --reps 10 > "$OUT/varprof.log" 2>&1) || { tail -20 "$OUT/varprof.log"; exit 1; }
             C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
             (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/varpmc" -o k -- python3 "$ROOT/tools/varpath_crossover.py" --reps 3 > "$OUT/varpmc.log" 2>&1) || { tail -20 "$OUT/varpmc.log"; exit 1; }
             python3 tools/pmc_summary.py "$OUT/varpmc" crc32c_chunk_kernel crc32c_finalize_kernel crc32c_direct_kernel plan_ sorted_ | tee "$OUT/varpmc.out"
             find "$OUT/varprof" -name '*kernel_stats.csv' -exec cp {} "$OUT/varprof_kernel_stats.csv" \;
             rm -rf "$OUT/varprof" "$OUT/varpmc" ;;
    flushprof) (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/flushprof" -o k -- "$ROOT/tools/flush_probe" 100 > "$OUT/flushprof.log" 2>&1) || { tail -20 "$OUT/flushprof.log"; exit 1; }
             cp "$OUT"/flushprof/*/k_kernel_stats.csv "$OUT/flushprof_kernel_stats.csv" 2>/dev/null || find "$OUT/flushprof" -name '*kernel_stats.csv' -exec cp {} "$OUT/flushprof_kernel_stats.csv" \;
             C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
             (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d "$OUT/flushpmc" -o k -- "$ROOT/tools/flush_probe" 20 > "$OUT/flushpmc.log" 2>&1) || { tail -20 "$OUT/flushpmc.log"; exit 1; }
             python3 tools/pmc_summary.py "$OUT/flushpmc" direct | tee "$OUT/flushpmc.out"
             rm -rf "$OUT/flushprof" "$OUT/flushpmc" ;;
    rehearsal) run bench_n2_rehearsal 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --share-device --steps 5 --warmup 2 --no-cpu ;;
    dlog) run bench_dlog 400 python bench.py --config dlog --steps 30 ;;
    latency) run latency_probe 300 env MI_CRC32C_GPU_MIN=0 python3 tools/latency_probe.py ;;
    zipf) run zipf_probe 300 python3 tools/zipf_probe.py ;;
    fixed) run fixed_probe 300 python3 tools/perf_probe.py ;;
    bench) run bench_default 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    shortab) for rnd in 1 2 3; do for v in 0 256 1024 4096; do
               echo -n "round $rnd short=$v "; MI_CRC32C_SORT_SHORT=$v timeout -k 10 120 python3 tools/zipf_probe.py > "$OUT/z.out" 2>&1 || { cat "$OUT/z.out"; exit 1; }; tail -1 "$OUT/z.out"
             done; done | tee "$OUT/shortab.out" ;;
    shortiso) for rnd in 1 2; do for cfg in "0 -" "1024 -" "256 -" "1024 keep" "0 keep" "0 drop" "1024 drop"; do
               set -- $cfg; v=$1; m=$2; envs="MI_CRC32C_SORT_SHORT=$v"
               [ "$m" = keep ] && envs="$envs ZIPF_KEEP_BELOW=1024"; [ "$m" = drop ] && envs="$envs ZIPF_DROP_BELOW=1024"
               echo -n "round $rnd short=$v class=$m "; env $envs timeout -k 10 120 python3 tools/zipf_probe.py > "$OUT/z.out" 2>&1 || { cat "$OUT/z.out"; exit 1; }; tail -1 "$OUT/z.out"
             done; done | tee "$OUT/shortiso.out" ;;
    laneab) for rnd in 1 2 3; do for v in 0 1 2 3; do
               echo -n "round $rnd lane_rows=$v "; MI_CRC32C_SORT_LANE_ROWS=$v timeout -k 10 120 python3 tools/zipf_probe.py > "$OUT/z.out" 2>&1 || { cat "$OUT/z.out"; exit 1; }; tail -1 "$OUT/z.out"
             done; done | tee "$OUT/laneab.out" ;;
    lanekeep) for rnd in 1 2; do for k in 257 1024; do for v in 0 2 3; do
               echo -n "round $rnd keep<$k lane_rows=$v "; ZIPF_KEEP_BELOW=$k MI_CRC32C_SORT_LANE_ROWS=$v timeout -k 10 120 python3 tools/zipf_probe.py > "$OUT/z.out" 2>&1 || { cat "$OUT/z.out"; exit 1; }; tail -1 "$OUT/z.out"
             done; done; done | tee "$OUT/lanekeep.out" ;;
    lanepmc) C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
             for v in 0 2; do
               envs="ZIPF_WARM=2 ZIPF_ROUNDS=1 ZIPF_KEEP_BELOW=257 MI_CRC32C_SORT_LANE_ROWS=$v"
               (cd /tmp && env $envs timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_l$v" -o k -- python3 "$ROOT/tools/zipf_probe.py" > "$OUT/pmc_l$v.log" 2>&1) || { tail -5 "$OUT/pmc_l$v.log"; exit 1; }
               echo "== keep<257 lane_rows=$v"; python3 tools/pmc_summary.py "$OUT/pmc_l$v" crc32c_sorted_kernel
             done | tee "$OUT/lanepmc.out" ;;
    lanetests) run pytest_lane 600 python -u -m pytest tests/test_gpu_sorted.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread ;;
    zipfpmc) C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
             for m in full keep drop; do
               envs="ZIPF_WARM=2 ZIPF_ROUNDS=1 MI_CRC32C_SORT_PIECE_LOG2=16 MI_CRC32C_SORT_RING=2"; [ "$m" = keep ] && envs="$envs ZIPF_KEEP_BELOW=1024"; [ "$m" = drop ] && envs="$envs ZIPF_DROP_BELOW=1024"
               (cd /tmp && env $envs timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$m" -o k -- python3 "$ROOT/tools/zipf_probe.py" > "$OUT/pmc_$m.log" 2>&1) || { tail -5 "$OUT/pmc_$m.log"; exit 1; }
               echo "== $m"; python3 tools/pmc_summary.py "$OUT/pmc_$m" crc32c_sorted_kernel sorted_cost_kernel
             done | tee "$OUT/zipfpmc.out" ;;
    direct) run pytest_direct 400 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_parity.py tests/test_durable_log.py -x -q --timeout 120 --timeout-method thread ;;
    sorted) run pytest_sorted 600 python -u -m pytest tests/test_gpu_sorted.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread ;;
    ab) AB_ROUNDS=${AB_ROUNDS:-3} run ab 900 python3 -u tools/ab.py --zipf "$@"; break ;;
    abfixed) AB_ROUNDS=${AB_ROUNDS:-3} run abfixed 900 python3 -u tools/ab.py "$@"; break ;;
    # kernel stats of the shipped build: the headline and configs[2] (sorted path)
    profhead) for cfg in fixed4k zipf; do
               (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$cfg" -o k -- python3 "$ROOT/bench.py" --config $cfg --steps 20 --warmup 5 --no-cpu --no-pmc --no-legs --sustain-seconds 0 > "$OUT/prof_$cfg.log" 2>&1) || { tail -20 "$OUT/prof_$cfg.log"; exit 1; }
               find "$OUT/prof_$cfg" -name '*kernel_stats.csv' -exec cp {} "$OUT/${cfg}_kernel_stats.csv" \;
               tail -1 "$OUT/prof_$cfg.log" > "$OUT/${cfg}_bench_under_prof.json"
               rm -rf "$OUT/prof_$cfg"; head -6 "$OUT/${cfg}_kernel_stats.csv"
             done ;;
    zc) run zc_probe 120 python3 tools/zc_probe.py ;;
    mid) for pth in pieces sorted; do run mid_$pth 300 python3 -u tools/mid_probe.py --path $pth --mib ${MID_MIB:-1,4,16,64,256} --reps 200 || exit 1; done ;;
    piecesweep) for rnd in 1 2; do for pl in ${SWEEP_PLOG:-13 14 15 16}; do for rg in ${SWEEP_RING:-4 2}; do
               MI_CRC32C_SORT_PIECE_LOG2=$pl MI_CRC32C_SORT_RING=$rg timeout -k 10 120 python3 tools/mid_probe.py --path sorted --mib ${MID_MIB:-128,256,512} --reps 100 > "$OUT/w.out" 2>&1 || { cat "$OUT/w.out"; exit 1; }; grep -v "^path" "$OUT/w.out" | sed "s/^/round $rnd plog=$pl ring=$rg /"
             done; done; done | tee "$OUT/piecesweep.out" ;;
    zipfenv) for rnd in 1 2 3 4; do for e in ${ZENV:-NONE=1}; do
               r=$(env ${e//,/ } timeout -k 10 120 python3 tools/zipf_probe.py consus_amd/lib/libconsus_crc32c.so 2>&1 | tail -1) || { echo "$r"; exit 1; }
               echo "round $rnd $e $r"; case "$r" in *MISMATCH*) exit 1;; esac
             done; done | tee "$OUT/zipfenv.out" ;;
    midenv) for rnd in 1 2; do for e in ${MENV:-NONE=1}; do
               env ${e//,/ } timeout -k 10 120 python3 tools/mid_probe.py --mib ${MID_MIB:-64,128,256} --reps 200 > "$OUT/w.out" 2>&1 || { cat "$OUT/w.out"; exit 1; }; grep -v "^path" "$OUT/w.out" | sed "s/^/round $rnd $e /"
             done; done | tee "$OUT/midenv.out" ;;
    smallrec) for rnd in 1 2; do for cfg in ${SMALLREC_CFGS:-engine_0_0 window_0_0 window_768_4 window_256_4 sorted_0_0}; do
               set -- ${cfg//_/ }; p=$1; [ "$p" = engine ] && p=""
               env MI_CRC32C_WIN_MAX_COUNT=16384 $( [ "$2" != 0 ] && echo MI_CRC32C_WIN_BLOCK=$2 ) $( [ "$3" != 0 ] && echo MI_CRC32C_WIN_ROWS=$3 ) timeout -k 10 120 python3 tools/mid_probe.py ${p:+--path $p} --uniform 42,1024 --mib ${MID_MIB:-1,2,4,6,8} --reps 200 > "$OUT/w.out" 2>&1 || { cat "$OUT/w.out"; exit 1; }; grep -v "^path" "$OUT/w.out" | sed "s/^/round $rnd $cfg /"
             done; done | tee "$OUT/smallrec.out" ;;
    adaptab) for rnd in 1 2 3 4; do for cfg in ${ADAPT_SET:-head:1 head:0}; do
               v=${cfg%%:*}; a=${cfg##*:}; lib=tools/ab/libconsus_crc32c_$v.so; [ "$v" = head ] && lib=consus_amd/lib/libconsus_crc32c.so
               r=$(MI_CRC32C_SORT_ADAPT=$a timeout -k 10 120 python3 tools/zipf_probe.py $lib 2>&1 | tail -1) || { echo "$r"; exit 1; }
               echo "round $rnd $v adapt=$a $r"; case "$r" in *MISMATCH*) exit 1;; esac
             done; done | tee "$OUT/adaptab.out" ;;
    winfetch) C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
             for m in ${WIN_MIB:-1 16 20}; do
               (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/wf_$m" -o k -- python3 "$ROOT/tools/mid_probe.py" --mib $m --reps 20 > "$OUT/wf_$m.log" 2>&1) || { tail -20 "$OUT/wf_$m.log"; exit 1; }
               echo "== $m MiB"; python3 tools/pmc_summary.py "$OUT/wf_$m" window_kernel; rm -rf "$OUT/wf_$m"
             done | tee "$OUT/winfetch.out" ;;
    winattr) C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
             for v in ${WINATTR_LIBS:-head winskip2 winskip7}; do
               lib=tools/ab/libconsus_crc32c_$v.so; [ "$v" = head ] && lib=consus_amd/lib/libconsus_crc32c.so
               for m in ${WIN_MIB:-16}; do
                 (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/wa_${v}_$m" -o k -- python3 "$ROOT/tools/mid_probe.py" --lib "$ROOT/$lib" --path window --mib $m --reps 20 > "$OUT/wa_${v}_$m.log" 2>&1) || { tail -20 "$OUT/wa_${v}_$m.log"; exit 1; }
                 echo "== $v $m MiB"; python3 tools/pmc_summary.py "$OUT/wa_${v}_$m" window_kernel; rm -rf "$OUT/wa_${v}_$m"
                 (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/wb_${v}_$m" -o k -- python3 "$ROOT/tools/mid_probe.py" --lib "$ROOT/$lib" --path window --mib $m --reps 20 > "$OUT/wb_${v}_$m.log" 2>&1) || { tail -20 "$OUT/wb_${v}_$m.log"; exit 1; }
                 python3 tools/pmc_summary.py "$OUT/wb_${v}_$m" window_kernel; rm -rf "$OUT/wb_${v}_$m"
               done
             done | tee "$OUT/winattr.out" ;;
    winprof) for m in ${WIN_MIB:-1 16 20}; do
               (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wp_$m" -o k -- python3 "$ROOT/tools/mid_probe.py" --mib $m --reps 100 > "$OUT/wp_$m.log" 2>&1) || { tail -20 "$OUT/wp_$m.log"; exit 1; }
               find "$OUT/wp_$m" -name '*kernel_stats.csv' -exec cp {} "$OUT/window_${m}mib_kernel_stats.csv" \;
               rm -rf "$OUT/wp_$m"; echo "== $m MiB"; grep -v "^path" "$OUT/wp_$m.log" | tail -2; head -3 "$OUT/window_${m}mib_kernel_stats.csv" | cut -c1-200
               (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/wpm_$m" -o k -- python3 "$ROOT/tools/mid_probe.py" --mib $m --reps 20 > "$OUT/wpm_$m.log" 2>&1) || { tail -20 "$OUT/wpm_$m.log"; exit 1; }
               echo "== $m MiB FETCH_SIZE (KiB, per dispatch, median; x2 gfx950 correction not applied)"; python3 tools/pmc_summary.py "$OUT/wpm_$m" window_kernel; rm -rf "$OUT/wpm_$m"
             done | tee "$OUT/winprof.out" ;;
    midprof) for pth in ${MID_PATHS:-pieces sorted}; do
               (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/midprof_$pth" -o k -- python3 "$ROOT/tools/mid_probe.py" --path $pth --mib ${MID_MIB:-64} --reps 50 > "$OUT/midprof_$pth.log" 2>&1) || { tail -20 "$OUT/midprof_$pth.log"; exit 1; }
               find "$OUT/midprof_$pth" -name '*kernel_trace.csv' -exec python3 "$ROOT/tools/kernel_gaps.py" {} 300 \; > "$OUT/midprof_${pth}_trace.txt" 2>&1
               rm -rf "$OUT/midprof_$pth"; cat "$OUT/midprof_${pth}_trace.txt"
             done ;;
    piecesweep) for pl in ${PLOGS:-16 14 13 12 11}; do MI_CRC32C_SORT_PIECE_LOG2=$pl run mid_sorted_p$pl 300 python3 -u tools/mid_probe.py --path sorted --mib ${MID_MIB:-16,64,256} --reps 100 || exit 1; done ;;
    ringsweep) for rg in ${RINGS:-2 4}; do MI_CRC32C_SORT_RING=$rg run mid_sorted_ring$rg 300 python3 -u tools/mid_probe.py --path sorted --mib ${MID_MIB:-1,4,16,64,256,512,1024,2048} --reps 100 || exit 1; done ;;
    stops) for rnd in 1 2; do for v in ${STOPS:-stop1 stop2 stop3 stop4 stop5 stop6 full}; do timeout -k 10 120 python3 -u tools/mid_probe.py --path sorted --mib ${MID_MIB:-1,64,256} --reps 100 --lib tools/ab/libconsus_crc32c_$v.so 2>&1 | grep -v "MiB" || exit 1; done; done | tee "$OUT/stops.out" ;;
    headab) cp consus_amd/lib/libconsus_crc32c.so tools/ab/libconsus_crc32c_r04.so && PERF_WARM=300 PERF_N=200 AB_ROUNDS=${AB_ROUNDS:-4} run headab 600 python3 -u tools/ab.py tools/ab/libconsus_crc32c_r02.so tools/ab/libconsus_crc32c_r03.so tools/ab/libconsus_crc32c_r04.so && cat "$OUT/headab.out" ;;
    piece4) for pl in 10 11 12 13; do MI_CRC32C_SORT_RING=4 MI_CRC32C_SORT_PIECE_LOG2=$pl run mid_sorted_r4p$pl 300 python3 -u tools/mid_probe.py --path sorted --mib ${MID_MIB:-1,16,64,256} --reps 100 || exit 1; done ;;
    fetchab) for v in ${FETCH_LIBS:-base edge}; do
               (cd /tmp && ZIPF_WARM=2 ZIPF_ROUNDS=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_$v" -o k -- python3 "$ROOT/tools/zipf_probe.py" "$ROOT/tools/ab/libconsus_crc32c_$v.so" > "$OUT/fetch_$v.log" 2>&1) || { tail -5 "$OUT/fetch_$v.log"; exit 1; }
               echo "== $v (FETCH_SIZE KB x2 per dispatch, median)"; python3 tools/pmc_summary.py "$OUT/fetch_$v" crc32c_sorted_kernel sorted_cost_kernel; rm -rf "$OUT/fetch_$v"
             done | tee "$OUT/fetchab.out" ;;
    fusedab) for fz in 1 0; do MI_CRC32C_SORT_FUSED=$fz run mid_fused$fz 300 python3 -u tools/mid_probe.py --path sorted --mib ${MID_MIB:-1,4,16,64,256} --reps 100 || exit 1; done ;;
    zipfring) for rnd in 1 2 3; do for rg in 2 4; do echo -n "round $rnd ring $rg "; MI_CRC32C_SORT_RING=$rg timeout -k 10 120 python3 tools/zipf_probe.py > "$OUT/z.out" 2>&1 || { cat "$OUT/z.out"; exit 1; }; tail -1 "$OUT/z.out"; done; done | tee "$OUT/zipfring.out" ;;
    # round 5: the records' shared 128-B lines (ZIPF_ALIGN=128 starts every
    # record on its own line; wrong digest by design), per library in tools/ab
    align) for rnd in 1 2; do for al in 0 128; do for lib in ${ALIGN_LIBS:-r04}; do
               echo -n "round $rnd align=$al $lib "; ZIPF_ALIGN=$al timeout -k 10 120 python3 tools/zipf_probe.py tools/ab/libconsus_crc32c_$lib.so > "$OUT/z.out" 2>&1 || { cat "$OUT/z.out"; exit 1; }; tail -1 "$OUT/z.out"
             done; done; done | tee "$OUT/align.out" ;;
    gpusorted) run pytest_sorted 900 python -u -m pytest tests/test_gpu_sorted.py tests/test_gpu_parity.py tests/test_gpu_errors.py tests/test_gpu_direct.py -x -q --timeout 120 --timeout-method thread ;;
    stamps) for m in ${STAMP_MIB:-0 256 1}; do echo "== mib $m"; timeout -k 10 120 python3 tools/sort_stamps.py tools/ab/libconsus_crc32c_${STAMP_LIB:-stamp}.so --mib $m ${STAMP_ARGS:-} || exit 1; done | tee "$OUT/stamps.out" ;;
    zipffused) for rnd in 1 2 3; do for fz in 1 0; do echo -n "round $rnd fused=$fz "; MI_CRC32C_SORT_FUSED=$fz timeout -k 10 120 python3 tools/zipf_probe.py > "$OUT/z.out" 2>&1 || { cat "$OUT/z.out"; exit 1; }; tail -1 "$OUT/z.out"; done; done | tee "$OUT/zipffused.out" ;;
    legcmp) for rnd in 1 2; do for k in 20 100; do
               echo -n "round $rnd bench --config zipf --steps $k (ms_per_step, events, sustained, digest): "; timeout -k 10 200 python3 bench.py --config zipf --steps $k --warmup 100 --no-cpu --no-pmc --leg-sustain-seconds 1 > "$OUT/lc.out" 2>"$OUT/lc.err" || { tail -5 "$OUT/lc.err"; exit 1; }
               python3 -c "import json,sys; r=json.loads(open('$OUT/lc.out').read().strip().splitlines()[-1]); print(r['ms_per_step'], r['roofline']['step_ms_events'], r['sustained']['step_ms'], r['digest_verified'])"
             done
             echo -n "round $rnd zipf_probe: "; timeout -k 10 120 python3 tools/zipf_probe.py > "$OUT/z.out" 2>&1 || { cat "$OUT/z.out"; exit 1; }; tail -1 "$OUT/z.out"
             done | tee "$OUT/legcmp.out" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "ALL OK"
