V=$PWD/build/var
bash tools/gpu_session.sh \
 "var:400:bash tools/variants_run.sh a1=UPE_GPU_LIB_DIAG=$V/a1.so a2=UPE_GPU_LIB_DIAG=$V/a2.so a4=UPE_GPU_LIB_DIAG=$V/a4.so a8=UPE_GPU_LIB_DIAG=$V/a8.so a15=UPE_GPU_LIB_DIAG=$V/a15.so a64=UPE_GPU_LIB_DIAG=$V/a64.so"
