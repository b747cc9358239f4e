# round 2: mid-chunk window prefetch issued after the chunk's output stores (UPE_MID_AT=3:
# the loop-top wait for it no longer waits for younger stores) against after the rule match
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix"
T="-m gpu -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh \
 "B0:120:python bench.py $O" \
 "Bat3:120:UPE_GPU_LIB_DIAG=$V/at3.so python bench.py $O" \
 "C0:120:python bench.py --config C $O" \
 "Cat3:120:UPE_GPU_LIB_DIAG=$V/at3.so python bench.py --config C $O" \
 "B0b:120:python bench.py $O" \
 "Bat3b:120:UPE_GPU_LIB_DIAG=$V/at3.so python bench.py $O" \
 "C0b:120:python bench.py --config C $O" \
 "Cat3b:120:UPE_GPU_LIB_DIAG=$V/at3.so python bench.py --config C $O" \
 "at3t:300:UPE_GPU_LIB_DIAG=$V/at3.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_neigh_paths.py $T"
