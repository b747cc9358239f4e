V=$PWD/build/var
bash tools/gpu_session.sh \
 "errors:200:python -u -m pytest tests/test_gpu_errors.py -x -v --timeout 120 --timeout-method thread" \
 "D:200:python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Dhr4096:200:UPE_GPU_LIB_DIAG=$V/hr4096.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Dhr2048:200:UPE_GPU_LIB_DIAG=$V/hr2048.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3"
