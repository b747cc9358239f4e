#!/bin/bash
# tree_probe over diagnostic builds: tools/r05_var.sh <cases> -- <lib.so>...
cases=""; while [ "$1" != "--" ]; do cases="$cases $1"; shift; done; shift
for lib in "$@"; do
  UPE_GPU_LIB_DIAG=$PWD/$lib timeout -k 10 200 python -u tools/tree_probe.py --steps 40 --out gpurun_out/var_$(basename $lib .so).jsonl $cases > gpurun_out/var_$(basename $lib .so).log 2>&1 || { echo "fail $lib"; exit 1; }
  echo "$lib: $(python -c "import json,sys; print([(r['case'], r['kernel_us']) for r in map(json.loads, open('gpurun_out/var_$(basename $lib .so).jsonl'))])")"
done
