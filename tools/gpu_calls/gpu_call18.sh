bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "benchB:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py --config B" \
 "benchC:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o p --output-format csv -- python bench.py --config C --no-cpu-baseline" \
 "benchD:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o p --output-format csv -- python bench.py --config D --steps 20 --warmup 2 --no-cpu-baseline --max-copies 4 --host-reps 3" \
 "pmcB:300:bash tools/pmc_run.sh B fetch write" \
 "pmcC:300:bash tools/pmc_run.sh C fetch write"
