# round 2, after the tuple-space probe changes: tests, PMC traffic for B / C / D (emit) written
# into profiles/ on the box before the bench lines read it, kernel-trace stats, bench lines
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "pmcB:300:bash tools/pmc_run.sh B emit fetch write && python tools/pmc_traffic.py B 1048576 emit" \
 "pmcC:300:bash tools/pmc_run.sh C emit fetch write && python tools/pmc_traffic.py C 1048576 emit" \
 "pmcD:300:bash tools/pmc_run.sh D emit fetch write sq sq2 && python tools/pmc_traffic.py D 16777216 emit" \
 "savepmc:30:mkdir -p gpurun_out/pmc_json && cp profiles/pmc_config*_emit.json gpurun_out/pmc_json/" \
 "benchB:400:python bench.py --host-reps 10 > gpurun_out/benchB.json" \
 "profB:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py --no-cpu-baseline --no-hbm-probe" \
 "profC:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o p --output-format csv -- python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "profD:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o p --output-format csv -- python bench.py --config D --no-cpu-baseline --no-hbm-probe --max-copies 4" \
 "benchC:300:python bench.py --config C --no-cpu-baseline > gpurun_out/benchC.json" \
 "benchD:300:python bench.py --config D --no-cpu-baseline --max-copies 4 > gpurun_out/benchD.json"
