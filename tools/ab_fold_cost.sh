#!/bin/bash
# dev A/B (round 5): sorted-path cost allowance per item (MI_SORT_FOLD_COST builds)
mkdir -p gpurun_out/r05an
for rnd in 1 2 3; do for L in fc2 fc1 fc3; do
  echo -n "round $rnd lib=$L "
  timeout -k 10 120 python3 tools/zipf_probe.py tools/ab/libconsus_crc32c_$L.so > gpurun_out/z.out 2>&1 || { cat gpurun_out/z.out; exit 1; }; tail -1 gpurun_out/z.out
done; done | tee gpurun_out/r05an/fc.out
