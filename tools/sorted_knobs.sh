set -o pipefail
AB_ROUNDS=3 timeout -k 10 900 python tools/ab.py --zipf tools/ab/libconsus_crc32c_m00.so tools/ab/libconsus_crc32c_m21.so tools/ab/libconsus_crc32c_m32.so tools/ab/libconsus_crc32c_m43.so tools/ab/libconsus_crc32c_m53.so
