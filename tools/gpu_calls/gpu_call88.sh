V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --host-reps 0"
bash tools/gpu_session.sh \
 "t1t:300:UPE_GPU_LIB_DIAG=$V/t1.so python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "B0:120:python bench.py $O" \
 "Bt1:120:UPE_GPU_LIB_DIAG=$V/t1.so python bench.py $O" \
 "Bt32:120:UPE_GPU_LIB_DIAG=$V/t32.so python bench.py $O" \
 "B0b:120:python bench.py $O" \
 "Bt1b:120:UPE_GPU_LIB_DIAG=$V/t1.so python bench.py $O" \
 "Bt32b:120:UPE_GPU_LIB_DIAG=$V/t32.so python bench.py $O"
