# round 2 profiles: default bench line (B, emit, cpu_baseline, host round trip), kernel-trace
# stats for B / C / D, PMC traffic for B / C / D in emit mode, stamps
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "benchB:400:python bench.py --host-reps 10 > gpurun_out/benchB.json" \
 "profB:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py --no-cpu-baseline --no-hbm-probe" \
 "profC:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o p --output-format csv -- python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "profD:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o p --output-format csv -- python bench.py --config D --no-cpu-baseline --no-hbm-probe --max-copies 4" \
 "pmcB:300:bash tools/pmc_run.sh B emit fetch write" \
 "pmcC:300:bash tools/pmc_run.sh C emit fetch write" \
 "pmcD:300:bash tools/pmc_run.sh D emit fetch write" \
 "stampsB:120:UPE_GPU_LIB_DIAG=\$PWD/build/var/stamps.so python tools/stamps.py 1048576 emit B > gpurun_out/stampsB.txt" \
 "stampsC:120:UPE_GPU_LIB_DIAG=\$PWD/build/var/stamps.so python tools/stamps.py 1048576 emit C > gpurun_out/stampsC.txt" \
 "benchC:300:python bench.py --config C --no-cpu-baseline > gpurun_out/benchC.json" \
 "benchD:300:python bench.py --config D --no-cpu-baseline --max-copies 4 > gpurun_out/benchD.json"
