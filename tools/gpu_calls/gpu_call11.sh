bash tools/gpu_session.sh \
 "variants:600:bash tools/variants_run.sh a1=UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a1.so a2=UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a2.so a4=UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a4.so a8=UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a8.so a15=UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a15.so a64=UPE_GPU_LIB_DIAG=$PWD/build/ablate/libupe_gpu_a64.so" \
 "sweep:400:bash tools/size_sweep.sh"
