bash tools/gpu_session.sh \
 "sweep:400:bash tools/size_sweep.sh" \
 "variants:600:bash tools/variants_run.sh"
