bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "variants:600:bash tools/variants_run.sh w6=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_w6.so w5=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_w5.so w4=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_w4.so"
