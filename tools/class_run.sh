set -o pipefail
ZIPF_KEEP_BELOW=256 timeout -k 10 120 python tools/sorted_stamps.py tools/ab/libconsus_crc32c_stamp.so
