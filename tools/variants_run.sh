#!/bin/bash
# Diagnostic: bench the product build and the occupancy / ablation variants (config B) under
# rocprofv3 kernel tracing, so every variant's kernel durations come from the profiler.
set -e
run() {  # label, then env assignments for the variant
  local label=$1; shift
  env "$@" rocprofv3 --kernel-trace --stats -d gpurun_out/var/$label -o v --output-format csv -- \
    python bench.py --no-cpu-baseline > gpurun_out/var_$label.json 2> gpurun_out/var_$label.err
}
run default UPE_BENCH_EVENTS=1
run noev UPE_BENCH_EVENTS=0
for t in 512 1024; do run t$t UPE_GPU_LIB_DIAG=$PWD/build/occ/libupe_gpu_t$t.so; done
for a in 1 2 4 8 15 16 64; do run a$a UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a$a.so; done
