V=$PWD/build/var
bash tools/gpu_session.sh \
 "var:300:VARIANTS_NONE=1 bash tools/variants_run.sh prio=UPE_GPU_LIB_DIAG=$V/prio.so" \
 "C:100:python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Cprio:100:UPE_GPU_LIB_DIAG=$V/prio.so python bench.py --config C --no-cpu-baseline --no-hbm-probe"
