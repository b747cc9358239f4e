#!/bin/bash
# Diagnostic build of libupe_gpu with extra -D flags: tools/build_variant.sh <out.so> [-DX=Y ...]
set -e
out=$1; shift
tmp=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" \
  -c -o $tmp/g.o upe_amd/csrc/upe_gpu.hip
mkdir -p $(dirname $out)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $tmp/g.o build/upe_host.o
rm -rf $tmp
