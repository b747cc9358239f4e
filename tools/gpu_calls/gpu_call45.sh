V=$PWD/build/var
bash tools/gpu_session.sh \
 "D:200:python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Da1:200:UPE_GPU_LIB_DIAG=$V/a1.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Da2:200:UPE_GPU_LIB_DIAG=$V/a2.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Da8:200:UPE_GPU_LIB_DIAG=$V/a8.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Da15:200:UPE_GPU_LIB_DIAG=$V/a15.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3"
