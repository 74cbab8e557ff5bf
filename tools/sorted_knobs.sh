set -o pipefail
AB_ROUNDS=5 timeout -k 10 900 python tools/ab.py tools/ab/libconsus_crc32c_tail0.so tools/ab/libconsus_crc32c_tail50.so tools/ab/libconsus_crc32c_tail100.so tools/ab/libconsus_crc32c_tail200.so
