bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "variants:600:bash tools/variants_run.sh g1w8=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_g1w8.so g1w6=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_g1w6.so g1w5=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_g1w5.so g0w8=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_g0w8.so g0w5=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_g0w5.so" \
 "testsC:300:UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_g1w5.so python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k 'golden or multi_batch or random_l1'"
