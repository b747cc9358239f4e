V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --host-reps 0"
bash tools/gpu_session.sh \
 "b512t:300:UPE_GPU_LIB_DIAG=$V/b512.so python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'golden_no_control or full_size_digest'" \
 "b512B:120:UPE_GPU_LIB_DIAG=$V/b512.so python bench.py $O" \
 "b512C:120:UPE_GPU_LIB_DIAG=$V/b512.so python bench.py --config C $O" \
 "b128t:300:UPE_GPU_LIB_DIAG=$V/b128.so python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'golden_no_control or full_size_digest'" \
 "b128B:120:UPE_GPU_LIB_DIAG=$V/b128.so python bench.py $O" \
 "b128C:120:UPE_GPU_LIB_DIAG=$V/b128.so python bench.py --config C $O" \
 "baseB:120:python bench.py $O"
