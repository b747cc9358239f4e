V=$PWD/build/var
bash tools/gpu_session.sh \
 "var:400:bash tools/variants_run.sh wperm=UPE_GPU_LIB_DIAG=$V/wperm.so" \
 "C:100:python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Cwperm:100:UPE_GPU_LIB_DIAG=$V/wperm.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "wpermt:200:UPE_GPU_LIB_DIAG=$V/wperm.so python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread"
