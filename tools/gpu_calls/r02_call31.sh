# round 2 (v11: lean emit kernel for launches without flow_hash / length side array / in-memory
# neighbour indexes): GPU tests, smoke, PMC traffic B / C emit, default bench line, rocprof of
# the default command split into legs, C and D lines with kernel stats
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "pmcB:300:bash tools/pmc_run.sh B emit fetch write && python tools/pmc_traffic.py B 1048576 emit" \
 "pmcC:300:bash tools/pmc_run.sh C emit fetch write && python tools/pmc_traffic.py C 1048576 emit" \
 "savepmc:30:mkdir -p gpurun_out/pmc_json && cp profiles/pmc_configB_emit.json profiles/pmc_configC_emit.json gpurun_out/pmc_json/" \
 "benchB:400:python bench.py --host-reps 10 > gpurun_out/benchB.json" \
 "profB:400:rocprofv3 --kernel-trace --stats -d gpurun_out/profB -o p --output-format csv -- python bench.py --no-cpu-baseline --no-hbm-probe" \
 "legs:60:python tools/kernel_legs.py gpurun_out/profB/p_kernel_trace.csv > gpurun_out/legsB.txt" \
 "benchC:300:python bench.py --config C --no-cpu-baseline > gpurun_out/benchC.json" \
 "profC:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o p --output-format csv -- python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "benchD:300:python bench.py --config D --no-cpu-baseline --max-copies 4 > gpurun_out/benchD.json"
