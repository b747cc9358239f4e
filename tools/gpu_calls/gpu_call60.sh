bash tools/gpu_session.sh \
 "profB:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py" \
 "profC:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o p --output-format csv -- python bench.py --config C" \
 "profD:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o p --output-format csv -- python bench.py --config D --no-cpu-baseline" \
 "pmcB:300:bash tools/pmc_run.sh B fetch write" \
 "pmcC:300:bash tools/pmc_run.sh C fetch write" \
 "pmcD:300:bash tools/pmc_run.sh D fetch write" \
 "hostB:300:python bench.py --host-reps 10 --no-cpu-baseline --no-hbm-probe" \
 "hostC:300:python bench.py --config C --host-reps 10 --no-cpu-baseline --no-hbm-probe" \
 "hostD:300:python bench.py --config D --steps 20 --warmup 2 --host-reps 3 --no-cpu-baseline --no-hbm-probe" \
 "C4M:200:python bench.py --config C --packets 4194304 --no-cpu-baseline --no-hbm-probe --steps 100" \
 "C16M:300:python bench.py --config C --packets 16777216 --no-cpu-baseline --no-hbm-probe --steps 20 --warmup 3"
