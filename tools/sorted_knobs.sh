#!/bin/bash
# A/B of sorted-path library builds on configs[2] (dev tool):
#   tools/build_variant.sh TAG -DMI_SORT_...=... ; tools/sorted_knobs.sh tools/ab/libconsus_crc32c_TAG.so ...
set -o pipefail
AB_ROUNDS=${AB_ROUNDS:-4} timeout -k 10 900 python tools/ab.py --zipf "$@"
