bash tools/gpu_session.sh \
 "stamps1M:200:UPE_GPU_LIB_DIAG=$PWD/build/diag/libupe_gpu_stamps.so python tools/stamps.py 1048576" \
 "stamps256k:200:UPE_GPU_LIB_DIAG=$PWD/build/diag/libupe_gpu_stamps.so python tools/stamps.py 262144"
