# round 2: lean tuple-space kernels (config D) against the previous build; parity of the
# tuple-space cases
V=$PWD/build/var
O="--config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3 --max-copies 4"
T="-m gpu -x -q --timeout 200 --timeout-method thread"
bash tools/gpu_session.sh \
 "Dprev:200:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py $O" \
 "Dlean:200:python bench.py $O" \
 "Dprevb:200:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py $O" \
 "Dleanb:200:python bench.py $O" \
 "dt:400:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py $T"
