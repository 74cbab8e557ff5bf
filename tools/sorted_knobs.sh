set -o pipefail
AB_ROUNDS=8 timeout -k 10 900 python tools/ab.py --zipf tools/ab/libconsus_crc32c_r2.so tools/ab/libconsus_crc32c_r4.so
