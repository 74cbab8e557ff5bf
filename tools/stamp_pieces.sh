set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r06s
for pl in 12 13 14 16; do
  echo "== piece 2^$pl"
  MI_CRC32C_SORT_PIECE_LOG2=$pl timeout -k 10 120 python3 tools/sort_stamps.py tools/ab/libconsus_crc32c_stamp.so --mib 256 | grep -v "^  e\|^  b\|^  r" || exit 1
done | tee gpurun_out/r06s/stamps_pieces.out
