bash tools/gpu_session.sh "pmc:600:bash tools/pmc_run.sh B sq sq2 sq3"
