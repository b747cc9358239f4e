V=$PWD/build/var
bash tools/gpu_session.sh \
 "var:400:bash tools/variants_run.sh pipe4=UPE_GPU_LIB_DIAG=$V/pipe4.so pipe5=UPE_GPU_LIB_DIAG=$V/pipe5.so" \
 "C:100:python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Cpipe4:100:UPE_GPU_LIB_DIAG=$V/pipe4.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Cpipe5:100:UPE_GPU_LIB_DIAG=$V/pipe5.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Cpipe4t:200:UPE_GPU_LIB_DIAG=$V/pipe4.so python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread"
