# round 2: first chunk's windows issued under the prologue's LDS staging (UPE_EARLY_WIN 1: staged
# items held in registers while the windows are issued; 2: windows issued after the LDS writes,
# before a bare barrier), against the product build, B and C, then parity of both variants
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode"
bash tools/gpu_session.sh \
 "def_B:120:python bench.py $O" \
 "ew1_B:120:UPE_GPU_LIB_DIAG=$V/ew1.so python bench.py $O" \
 "ew2_B:120:UPE_GPU_LIB_DIAG=$V/ew2.so python bench.py $O" \
 "def_C:120:python bench.py --config C $O" \
 "ew1_C:120:UPE_GPU_LIB_DIAG=$V/ew1.so python bench.py --config C $O" \
 "ew2_C:120:UPE_GPU_LIB_DIAG=$V/ew2.so python bench.py --config C $O" \
 "def_B2:120:python bench.py $O" \
 "ew1_B2:120:UPE_GPU_LIB_DIAG=$V/ew1.so python bench.py $O" \
 "ew2_B2:120:UPE_GPU_LIB_DIAG=$V/ew2.so python bench.py $O" \
 "def_D:200:python bench.py --config D --steps 30 --warmup 3 --max-copies 4 $O" \
 "ew1_D:200:UPE_GPU_LIB_DIAG=$V/ew1.so python bench.py --config D --steps 30 --warmup 3 --max-copies 4 $O" \
 "ew1t:300:UPE_GPU_LIB_DIAG=$V/ew1.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_neigh_paths.py tests/test_gpu_batches.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "ew2t:300:UPE_GPU_LIB_DIAG=$V/ew2.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_neigh_paths.py tests/test_gpu_batches.py -m gpu -x -q --timeout 120 --timeout-method thread"
