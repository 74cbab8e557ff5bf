#!/bin/bash
# Build an A/B variant of the engine library with extra -D flags (dev tool):
#   tools/build_variant.sh TAG -DFOO=1 ...   ->  tools/ab/libconsus_crc32c_TAG.so
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
TAG="$1"; shift
OUT="$ROOT/tools/ab"; mkdir -p "$OUT" "/tmp/abv_$TAG"
rm -f /tmp/abv_$TAG/*.o
SRC="$ROOT/consus_amd/csrc"
FL="-O3 -std=c++17 -fPIC -I$ROOT/include $*"
for f in crc32c_kernels.hip engine.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $FL -c -o /tmp/abv_$TAG/$f.o $SRC/$f &
done
for f in api.cc host_crc.cc durable_log.cc workload.cc; do
  g++ $FL -c -o /tmp/abv_$TAG/$f.o $SRC/$f &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libconsus_crc32c_$TAG.so" /tmp/abv_$TAG/*.o -lrccl -lpthread
echo "$OUT/libconsus_crc32c_$TAG.so"
