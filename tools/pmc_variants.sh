#!/bin/bash
# SQ instruction counters per ablation variant (config B), one rocprofv3 pass each.
set -e
for v in default a1 a2 a4 a8 a15; do
  if [ $v = default ]; then lib=""; else lib="UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_${v}.so"; fi
  env $lib rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
    -d gpurun_out/pmcv/$v -o p --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pmcv_$v.log 2>&1
  env $lib rocprofv3 --kernel-trace --stats -d gpurun_out/var/$v -o v --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err
done
