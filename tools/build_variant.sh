#!/bin/bash
# Diagnostic build of libupe_gpu with extra -D flags: tools/build_variant.sh <out.so> [-DX=Y ...]
# (timing experiments; the product library is built by `make -C upe_amd/csrc`)
set -e
out=$(realpath -m "$1"); shift
cd "$(dirname "$0")/.."
make -s -C upe_amd/csrc "$PWD/build/upe_host.o" "$PWD/build/upe_worker.o" >/dev/null
tmp=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" \
  -c -o $tmp/g.o upe_amd/csrc/upe_gpu.hip
mkdir -p "$(dirname "$out")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" $tmp/g.o build/upe_host.o build/upe_worker.o
rm -rf $tmp
