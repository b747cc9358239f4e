bash tools/gpu_session.sh \
 "profB:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py" \
 "profC:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o p --output-format csv -- python bench.py --config C" \
 "profD:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o p --output-format csv -- python bench.py --config D --no-cpu-baseline" \
 "hostD:300:python bench.py --config D --steps 20 --warmup 2 --host-reps 3 --no-cpu-baseline --no-hbm-probe" \
 "D64M:300:python bench.py --config D --packets 67108864 --steps 10 --warmup 2 --no-cpu-baseline --no-hbm-probe"
