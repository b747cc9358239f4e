V=$PWD/build/var
O="--config D --steps 20 --warmup 2 --max-copies 4 --no-cpu-baseline --no-hbm-probe --host-reps 0"
bash tools/gpu_session.sh \
 "base:200:python bench.py $O" \
 "r16k:200:UPE_GPU_LIB_DIAG=$V/r16k.so python bench.py $O" \
 "t4k:200:UPE_GPU_LIB_DIAG=$V/t4k.so python bench.py $O" \
 "t1k:200:UPE_GPU_LIB_DIAG=$V/t1k.so python bench.py $O" \
 "r16kt1k:200:UPE_GPU_LIB_DIAG=$V/r16kt1k.so python bench.py $O"
