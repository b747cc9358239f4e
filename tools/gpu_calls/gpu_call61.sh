V=$PWD/build/var
bash tools/gpu_session.sh \
 "var:300:VARIANTS_NONE=1 bash tools/variants_run.sh noinl=UPE_GPU_LIB_DIAG=$V/noinl.so noinl2=UPE_GPU_LIB_DIAG=$V/noinl.so def2=UPE_BENCH_EVENTS=1"
