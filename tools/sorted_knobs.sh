set -o pipefail
AB_ROUNDS=3 AB_ALLOW_MISMATCH=1 timeout -k 10 900 python tools/ab.py --zipf tools/ab/libconsus_crc32c_base.so tools/ab/libconsus_crc32c_ab4.so tools/ab/libconsus_crc32c_ab16.so tools/ab/libconsus_crc32c_ab20.so
