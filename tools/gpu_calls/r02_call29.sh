# round 2: SQ counters of the current kernel for configs B and C (emit), to see how busy the
# SIMDs' VALU is now that the window of the next chunk is prefetched
bash tools/gpu_session.sh \
 "pmcB:300:bash tools/pmc_run.sh B emit sq sq2 && python tools/pmc_summary.py B emit > gpurun_out/sqB.txt" \
 "pmcC:300:bash tools/pmc_run.sh C emit sq sq2 && python tools/pmc_summary.py C emit > gpurun_out/sqC.txt"
