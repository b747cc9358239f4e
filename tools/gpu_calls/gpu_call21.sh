bash tools/gpu_session.sh \
 "variants:600:bash tools/variants_run.sh w4=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_w4.so w6=UPE_GPU_LIB_DIAG=$PWD/build/var/libupe_gpu_w6.so" \
 "stamps1M:200:UPE_GPU_LIB_DIAG=$PWD/build/diag/libupe_gpu_stamps.so python tools/stamps.py 1048576" \
 "sweep:400:bash tools/size_sweep.sh"
