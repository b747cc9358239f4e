bash tools/gpu_session.sh \
 "benchB:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py --config B --no-cpu-baseline --host-reps 0" \
 "benchB2:300:python bench.py --config B --no-cpu-baseline --host-reps 0" \
 "benchC:300:python bench.py --config C --no-cpu-baseline --host-reps 0"
