# round 2: bench line with the IMIX leg (config C timed after the main region), its rocprof
# kernel trace split into legs, and a 2-rank rehearsal of the multi-GPU path on one GPU (gloo)
bash tools/gpu_session.sh \
 "bench:400:python bench.py > gpurun_out/bench_imix.json" \
 "prof:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profBI -o p --output-format csv -- python bench.py --no-cpu-baseline --no-hbm-probe" \
 "legs:60:python tools/kernel_legs.py gpurun_out/profBI/p_kernel_trace.csv > gpurun_out/legs.txt" \
 "rank2:400:UPE_BENCH_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 100 --warmup 10 --no-hbm-probe > gpurun_out/rank2.json"
