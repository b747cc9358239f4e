V=$PWD/build/var
bash tools/gpu_session.sh \
 "C:100:python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Ca2:100:UPE_GPU_LIB_DIAG=$V/a2.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Ca4:100:UPE_GPU_LIB_DIAG=$V/a4.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Ca8:100:UPE_GPU_LIB_DIAG=$V/a8.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Ca15:100:UPE_GPU_LIB_DIAG=$V/a15.so python bench.py --config C --no-cpu-baseline --no-hbm-probe" \
 "Ca64:100:UPE_GPU_LIB_DIAG=$V/a64.so python bench.py --config C --no-cpu-baseline --no-hbm-probe"
