#!/bin/bash
# config D with a diagnostic build vs the product library (tools/d_probe.py full)
for lib in "$@"; do
  if [ "$lib" = product ]; then env=""; else env="UPE_GPU_LIB_DIAG=$PWD/$lib"; fi
  env $env timeout -k 10 200 python tools/d_probe.py full --steps 12 2>&1 | grep classify || { echo "fail $lib"; exit 1; }
done
