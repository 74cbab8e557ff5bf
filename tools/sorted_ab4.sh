#!/bin/bash
# A/B of sorted-kernel build variants (dev tool): tools/ab.py --zipf over the
# libraries in tools/ab/, the full configs[2] step and the < 1 KiB class alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 9
mkdir -p gpurun_out/ab4
L="tools/ab/libconsus_crc32c_base.so $*"
echo "== full"; AB_ROUNDS=4 timeout -k 10 400 python3 -u tools/ab.py --zipf $L | tee gpurun_out/ab4/full.txt || exit 1
echo "== keep1024"; ZIPF_KEEP_BELOW=1024 MI_CRC32C_VARPATH=sorted AB_ALLOW_MISMATCH=1 AB_ROUNDS=3 timeout -k 10 300 python3 -u tools/ab.py --zipf $L | tee gpurun_out/ab4/keep.txt
