V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --host-reps 0"
bash tools/gpu_session.sh \
 "C0:120:python bench.py --config C $O" \
 "C1:120:UPE_GPU_LIB_DIAG=$V/ab1.so python bench.py --config C $O" \
 "C2:120:UPE_GPU_LIB_DIAG=$V/ab2.so python bench.py --config C $O" \
 "C4:120:UPE_GPU_LIB_DIAG=$V/ab4.so python bench.py --config C $O" \
 "C8:120:UPE_GPU_LIB_DIAG=$V/ab8.so python bench.py --config C $O" \
 "B0:120:python bench.py $O" \
 "B1:120:UPE_GPU_LIB_DIAG=$V/ab1.so python bench.py $O" \
 "B2:120:UPE_GPU_LIB_DIAG=$V/ab2.so python bench.py $O" \
 "B4:120:UPE_GPU_LIB_DIAG=$V/ab4.so python bench.py $O" \
 "B8:120:UPE_GPU_LIB_DIAG=$V/ab8.so python bench.py $O"
