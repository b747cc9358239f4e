V=$PWD/build/var
bash tools/gpu_session.sh \
 "var:300:VARIANTS_NONE=1 bash tools/variants_run.sh prev=UPE_GPU_LIB_DIAG=$V/prev.so" \
 "C:100:python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Cprev:100:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "C2:100:python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Cprev2:100:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "D:200:python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
