bash tools/gpu_session.sh \
 "profC4M:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profC4M -o p --output-format csv -- python bench.py --config C --packets 4194304 --no-cpu-baseline --no-hbm-probe --steps 100" \
 "profB16M:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profB16M -o p --output-format csv -- python bench.py --packets 16777216 --no-cpu-baseline --no-hbm-probe --steps 50 --warmup 5"
