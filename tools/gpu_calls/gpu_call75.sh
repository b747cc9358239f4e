V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --host-reps 0"
bash tools/gpu_session.sh \
 "base_B:120:python bench.py $O" \
 "w4_B:120:UPE_GPU_LIB_DIAG=$V/w4.so python bench.py $O" \
 "base_C:120:python bench.py --config C $O" \
 "w4_C:120:UPE_GPU_LIB_DIAG=$V/w4.so python bench.py --config C $O" \
 "base_D:200:python bench.py --config D --steps 20 --warmup 2 --max-copies 4 $O" \
 "w4_D:200:UPE_GPU_LIB_DIAG=$V/w4.so python bench.py --config D --steps 20 --warmup 2 --max-copies 4 $O"
