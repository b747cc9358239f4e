bash tools/gpu_session.sh \
 "pmcD:200:bash tools/pmc_run.sh D fetch write"
