V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --host-reps 0"
bash tools/gpu_session.sh \
 "base_B:120:python bench.py $O" \
 "ch3_B:120:UPE_GPU_LIB_DIAG=$V/ch3.so python bench.py $O" \
 "base_B2:120:python bench.py $O" \
 "ch3_B2:120:UPE_GPU_LIB_DIAG=$V/ch3.so python bench.py $O" \
 "base_B16:120:python bench.py --packets 16777216 --steps 40 $O" \
 "ch3_B16:120:UPE_GPU_LIB_DIAG=$V/ch3.so python bench.py --packets 16777216 --steps 40 $O"
