#!/bin/bash
# Diagnostic: bench the product build and diagnostic variants (config B) under rocprofv3 kernel
# tracing, so every variant's kernel durations come from the profiler.
#   tools/variants_run.sh [label=ENV=VALUE ...]   (default: ablation + grid variants)
set -e
run() {  # label, then env assignments for the variant
  local label=$1; shift
  env "$@" rocprofv3 --kernel-trace --stats -d gpurun_out/var/$label -o v --output-format csv -- \
    python bench.py --no-cpu-baseline > gpurun_out/var_$label.json 2> gpurun_out/var_$label.err
}
run default UPE_BENCH_EVENTS=1
run noev UPE_BENCH_EVENTS=0
if [ $# -eq 0 ] && [ -z "${VARIANTS_NONE:-}" ]; then
  set -- a2=UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a2.so \
         a4=UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a4.so \
         a15=UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a15.so \
         a64=UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a64.so \
         g4=UPE_GPU_BLOCKS_PER_CU=4 g16=UPE_GPU_BLOCKS_PER_CU=16
fi
for spec in "$@"; do run "${spec%%=*}" "${spec#*=}"; done
