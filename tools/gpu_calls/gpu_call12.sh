bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "variants:600:bash tools/variants_run.sh w8=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_w8.so w6=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_w6.so w4=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_w4.so" \
 "sweep:400:bash tools/size_sweep.sh"
