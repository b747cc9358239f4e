#!/bin/bash
# Diagnostic: config D under ablation builds (kernel durations from rocprofv3).
run() {
  local label=$1; shift
  env "$@" rocprofv3 --kernel-trace --stats -d gpurun_out/var/$label -o v --output-format csv -- \
    python bench.py --config D --steps 6 --warmup 1 --no-cpu-baseline --max-copies 2 --host-reps 0 > gpurun_out/var_$label.json 2> gpurun_out/var_$label.err
}
run default UPE_BENCH_EVENTS=1
for a in 1 2 4 8 15; do run a$a UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a$a.so; done
