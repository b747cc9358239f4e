#!/bin/bash
# Kernel duration vs batch size (config B), to separate per-round latency from bandwidth.
set -e
for n in 262144 524288 1048576 2097152 4194304; do
  rocprofv3 --kernel-trace --stats -d gpurun_out/sweep/n$n -o s --output-format csv -- \
    python bench.py --no-cpu-baseline --packets $n --max-copies 64 > gpurun_out/sweep_n$n.json 2> gpurun_out/sweep_n$n.err
done
