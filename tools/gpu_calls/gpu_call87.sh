V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --host-reps 0"
bash tools/gpu_session.sh \
 "B0:120:python bench.py $O" \
 "Bcwb:120:UPE_GPU_LIB_DIAG=$V/cwb.so python bench.py $O" \
 "B8:120:UPE_GPU_LIB_DIAG=$V/ab8.so python bench.py $O" \
 "C0:120:python bench.py --config C $O" \
 "Ccwb:120:UPE_GPU_LIB_DIAG=$V/cwb.so python bench.py --config C $O" \
 "C8:120:UPE_GPU_LIB_DIAG=$V/ab8.so python bench.py --config C $O"
