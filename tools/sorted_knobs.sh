set -o pipefail
timeout -k 10 120 python tools/sorted_stamps.py tools/ab/libconsus_crc32c_stampx20.so | grep -E "xcd|WG end|end  " && \
AB_ROUNDS=4 timeout -k 10 900 python tools/ab.py --zipf tools/ab/libconsus_crc32c_base.so tools/ab/libconsus_crc32c_xcd20.so tools/ab/libconsus_crc32c_xcd30.so tools/ab/libconsus_crc32c_xcd40.so
