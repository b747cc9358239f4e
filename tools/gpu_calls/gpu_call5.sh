rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
bash tools/gpu_session.sh "pmc:600:bash tools/pmc_run.sh B fetch write sq sq2 sq3 clk ta tcp tcc"
