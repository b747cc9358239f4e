bash tools/gpu_session.sh \
 "pmcB:300:bash tools/pmc_run.sh B fetch write" \
 "pmcC:300:bash tools/pmc_run.sh C fetch write" \
 "pmcD:300:bash tools/pmc_run.sh D fetch write"
