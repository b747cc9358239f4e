V=$PWD/build/var
bash tools/gpu_session.sh \
 "var:300:VARIANTS_NONE=1 bash tools/variants_run.sh early=UPE_GPU_LIB_DIAG=$V/early.so early2=UPE_GPU_LIB_DIAG=$V/early.so def2=UPE_BENCH_EVENTS=1" \
 "C:100:python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Cearly:100:UPE_GPU_LIB_DIAG=$V/early.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "D:200:python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Dearly:200:UPE_GPU_LIB_DIAG=$V/early.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "earlyt:300:UPE_GPU_LIB_DIAG=$V/early.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread"
