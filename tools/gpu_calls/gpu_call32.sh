bash tools/gpu_session.sh \
 "B4M:200:python bench.py --packets 4194304 --no-cpu-baseline --no-hbm-probe --steps 100" \
 "B16M:200:python bench.py --packets 16777216 --no-cpu-baseline --no-hbm-probe --steps 50 --warmup 5" \
 "C4M:200:python bench.py --config C --packets 4194304 --no-cpu-baseline --no-hbm-probe --steps 100" \
 "profD:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o p --output-format csv -- python bench.py --config D --no-cpu-baseline --no-hbm-probe"
