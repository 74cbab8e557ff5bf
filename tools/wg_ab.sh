#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/wg
for rnd in 1 2 3; do for w in 64 128 256; do
  echo "== round $rnd wg $w"
  LD_LIBRARY_PATH=$PWD/tools/ab/wg$w timeout -k 10 120 ./tools/flush_probe 500 > gpurun_out/wg/r${rnd}_$w.txt 2>&1 || { cat gpurun_out/wg/r${rnd}_$w.txt; exit 1; }
  cat gpurun_out/wg/r${rnd}_$w.txt
done; done
