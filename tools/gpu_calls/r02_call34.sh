# round 2 (v12, lean kernels for every config): GPU tests, smoke, driver-style and default bench
# lines, rocprof of the default command split into legs, C and D lines and kernel stats
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench20:300:python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20.json" \
 "benchB:400:python bench.py --host-reps 10 > gpurun_out/benchB.json" \
 "profB:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py --no-cpu-baseline --no-hbm-probe" \
 "legs:60:python tools/kernel_legs.py gpurun_out/profB/p_kernel_trace.csv > gpurun_out/legsB.txt" \
 "benchC:300:python bench.py --config C --no-cpu-baseline > gpurun_out/benchC.json" \
 "profC:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o p --output-format csv -- python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "benchD:300:python bench.py --config D --no-cpu-baseline --max-copies 4 > gpurun_out/benchD.json" \
 "profD:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o p --output-format csv -- python bench.py --config D --no-cpu-baseline --no-hbm-probe --max-copies 4"
