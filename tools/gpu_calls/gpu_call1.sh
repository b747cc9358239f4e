bash tools/gpu_session.sh \
 "tests:900:python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread" \
 "benchB:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py --config B" \
 "benchC:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o p --output-format csv -- python bench.py --config C --no-cpu-baseline" \
 "benchD:400:python bench.py --config D --steps 5 --warmup 1 --no-cpu-baseline --max-copies 2" \
 "pmcF:120:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcB_fetch -o p --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline" \
 "pmcW:120:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcB_write -o p --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline"
