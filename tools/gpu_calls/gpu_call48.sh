V=$PWD/build/var
bash tools/gpu_session.sh \
 "var:300:VARIANTS_NONE=1 bash tools/variants_run.sh gpi=UPE_GPU_LIB_DIAG=$V/gpi.so" \
 "C:100:python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Cgpi:100:UPE_GPU_LIB_DIAG=$V/gpi.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "D:200:python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Dgpi:200:UPE_GPU_LIB_DIAG=$V/gpi.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "gpit:300:UPE_GPU_LIB_DIAG=$V/gpi.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread"
