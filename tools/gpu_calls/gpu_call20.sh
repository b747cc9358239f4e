bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "variants:600:bash tools/variants_run.sh w4=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_w4.so w6=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_w6.so" \
 "stamps1M:200:UPE_GPU_LIB_DIAG=$PWD/build/diag/libupe_gpu_stamps.so python tools/stamps.py 1048576" \
 "benchC:300:python bench.py --config C --no-cpu-baseline"
