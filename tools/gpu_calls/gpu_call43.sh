V=$PWD/build/var
bash tools/gpu_session.sh \
 "C:100:python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Chist64:100:UPE_GPU_LIB_DIAG=$V/hist64.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "D:200:python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 50 --warmup 5" \
 "hist64t:300:UPE_GPU_LIB_DIAG=$V/hist64.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread" \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
