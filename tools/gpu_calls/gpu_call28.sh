V=$PWD/build/var
bash tools/gpu_session.sh \
 "var:400:bash tools/variants_run.sh fullwb=UPE_GPU_LIB_DIAG=$V/fullwb.so nt=UPE_GPU_LIB_DIAG=$V/nt.so fullnt=UPE_GPU_LIB_DIAG=$V/fullnt.so" \
 "C:100:python bench.py --config C --no-cpu-baseline" \
 "Cfullwb:100:UPE_GPU_LIB_DIAG=$V/fullwb.so python bench.py --config C --no-cpu-baseline" \
 "Cnt:100:UPE_GPU_LIB_DIAG=$V/nt.so python bench.py --config C --no-cpu-baseline" \
 "Cfullnt:100:UPE_GPU_LIB_DIAG=$V/fullnt.so python bench.py --config C --no-cpu-baseline"
