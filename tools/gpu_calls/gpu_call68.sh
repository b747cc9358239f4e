bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "profB:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py" \
 "profC:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o p --output-format csv -- python bench.py --config C" \
 "profD:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o p --output-format csv -- python bench.py --config D --no-cpu-baseline" \
 "pmcB:300:bash tools/pmc_run.sh B fetch write" \
 "pmcC:300:bash tools/pmc_run.sh C fetch write" \
 "pmcD:300:bash tools/pmc_run.sh D fetch write" \
 "hostB:300:python bench.py --host-reps 10 --no-cpu-baseline --no-hbm-probe" \
 "hostC:300:python bench.py --config C --host-reps 10 --no-cpu-baseline --no-hbm-probe" \
 "B4M:200:python bench.py --packets 4194304 --no-cpu-baseline --no-hbm-probe --steps 100" \
 "B16M:200:python bench.py --packets 16777216 --no-cpu-baseline --no-hbm-probe --steps 50 --warmup 5" \
 "C4M:200:python bench.py --config C --packets 4194304 --no-cpu-baseline --no-hbm-probe --steps 100" \
 "C16M:300:python bench.py --config C --packets 16777216 --no-cpu-baseline --no-hbm-probe --steps 20 --warmup 3"
