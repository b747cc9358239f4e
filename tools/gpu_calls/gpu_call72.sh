V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --host-reps 0"
bash tools/gpu_session.sh \
 "base_B:120:python bench.py $O" \
 "a0_B:120:UPE_GPU_LIB_DIAG=$V/a0.so python bench.py $O" \
 "a0w6_B:120:UPE_GPU_LIB_DIAG=$V/a0w6.so python bench.py $O" \
 "a0w8_B:120:UPE_GPU_LIB_DIAG=$V/a0w8.so python bench.py $O" \
 "w6_B:120:UPE_GPU_LIB_DIAG=$V/w6.so python bench.py $O" \
 "base_C:120:python bench.py --config C $O" \
 "a0w6_C:120:UPE_GPU_LIB_DIAG=$V/a0w6.so python bench.py --config C $O" \
 "w6_C:120:UPE_GPU_LIB_DIAG=$V/w6.so python bench.py --config C $O" \
 "a0w8_C:120:UPE_GPU_LIB_DIAG=$V/a0w8.so python bench.py --config C $O"
