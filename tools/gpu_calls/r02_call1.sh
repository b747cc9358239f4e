# round 2: tests, default bench (B, emit, with cpu_baseline), kernel-trace profile, PMC traffic,
# configs C and D
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "benchB:400:python bench.py > gpurun_out/benchB.json" \
 "profB:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py --no-cpu-baseline --host-reps 0" \
 "pmcB:300:bash tools/pmc_run.sh B emit fetch write" \
 "benchC:400:python bench.py --config C --no-cpu-baseline > gpurun_out/benchC.json" \
 "benchD:400:python bench.py --config D --no-cpu-baseline --max-copies 4 > gpurun_out/benchD.json"
