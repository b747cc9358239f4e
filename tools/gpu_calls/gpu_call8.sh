bash tools/gpu_session.sh "varD:600:bash tools/variants_d.sh"
