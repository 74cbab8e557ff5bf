set -o pipefail
mkdir -p gpurun_out/lay
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lay/gpu.txt 2>&1 || { tail -30 gpurun_out/lay/gpu.txt; exit 1; }
tail -1 gpurun_out/lay/gpu.txt
AB_ROUNDS=5 timeout -k 10 900 python tools/ab.py --zipf tools/ab/libconsus_crc32c_lold.so tools/ab/libconsus_crc32c_lnew.so
AB_ROUNDS=5 timeout -k 10 900 python tools/ab.py tools/ab/libconsus_crc32c_lold.so tools/ab/libconsus_crc32c_lnew.so
