# round 2 (v13, no-look-back kernels): smoke, driver-style and default bench lines, rocprof of
# the default command split into legs, C and D lines with kernel stats, 2-rank rehearsal
bash tools/gpu_session.sh \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench20:300:python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20.json" \
 "benchB:400:python bench.py --host-reps 10 > gpurun_out/benchB.json" \
 "profB:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py --no-cpu-baseline --no-hbm-probe" \
 "legs:60:python tools/kernel_legs.py gpurun_out/profB/p_kernel_trace.csv > gpurun_out/legsB.txt" \
 "benchC:300:python bench.py --config C --no-cpu-baseline > gpurun_out/benchC.json" \
 "profC:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o p --output-format csv -- python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "benchD:300:python bench.py --config D --no-cpu-baseline --max-copies 4 > gpurun_out/benchD.json" \
 "profD:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o p --output-format csv -- python bench.py --config D --no-cpu-baseline --no-hbm-probe --max-copies 4" \
 "rank2:400:UPE_BENCH_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29547 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/rank2.json"
