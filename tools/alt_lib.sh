#!/bin/bash
# Build an A/B copy of the codec library with extra compiler flags for the two
# LZ4 sources only (the rest linked from the normal build's objects):
#   bash tools/alt_lib.sh TAG -mllvm -some-flag ...  -> bitshuffle_amd/libbitshuffle_mi355x_TAG.so
set -e
TAG=$1; shift
cd "$(dirname "$0")/../bitshuffle_amd"
F="--offload-arch=gfx950 ${OPT:--O3} -std=c++17 -fPIC -Wall -I../include -Wno-unused-result -munsafe-fp-atomics -mllvm -structurizecfg-skip-uniform-regions"
mkdir -p /tmp/alt_$TAG
/opt/rocm/bin/hipcc $F "$@" -c csrc/lz4_encode.hip -o /tmp/alt_$TAG/lz4_encode.o &
/opt/rocm/bin/hipcc $F "$@" -c csrc/lz4_decode.hip -o /tmp/alt_$TAG/lz4_decode.o &
wait
objs=""
for o in build/*.o; do b=$(basename $o); [ -f /tmp/alt_$TAG/$b ] && objs="$objs /tmp/alt_$TAG/$b" || objs="$objs $o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libbitshuffle_mi355x_$TAG.so $objs -Wl,-z,nodelete
