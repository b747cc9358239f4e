#!/bin/bash
# A/B of diagnostic builds: config D (full table / frames-only), B, CF, C3 kernel times
for lib in "$@"; do
  b=$(basename $lib .so)
  for v in full small; do
    UPE_GPU_LIB_DIAG=$PWD/$lib timeout -k 10 200 python tools/d_probe.py $v > gpurun_out/ab_${b}_d$v.log 2>&1 || { echo "fail $lib d $v"; exit 1; }
    echo "$b D-$v $(grep classify gpurun_out/ab_${b}_d$v.log)"
  done
  UPE_GPU_LIB_DIAG=$PWD/$lib timeout -k 10 200 python -u tools/tree_probe.py --steps 40 --out gpurun_out/ab_$b.jsonl B:tree CF:tree C3:scan > gpurun_out/ab_$b.log 2>&1 || { echo "fail $lib probe"; exit 1; }
  echo "$b: $(python -c "import json; print([(r['case'], r['kernel_us']) for r in map(json.loads, open('gpurun_out/ab_$b.jsonl'))])")"
done
