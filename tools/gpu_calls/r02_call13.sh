# round 2: mid-chunk window prefetch placement (after the parse: AT=1; after the rule match:
# AT=2) and the in-place kernel (MID=3), B / C emit and B in place; parity of AT=1
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix"
T="-m gpu -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh \
 "B0:120:python bench.py $O" \
 "Bm1a2:120:UPE_GPU_LIB_DIAG=$V/m1a2.so python bench.py $O" \
 "Bm1a1:120:UPE_GPU_LIB_DIAG=$V/m1a1.so python bench.py $O" \
 "C0:120:python bench.py --config C $O" \
 "Cm1a2:120:UPE_GPU_LIB_DIAG=$V/m1a2.so python bench.py --config C $O" \
 "Cm1a1:120:UPE_GPU_LIB_DIAG=$V/m1a1.so python bench.py --config C $O" \
 "Bi0:120:python bench.py --mode inplace $O" \
 "Bim3:120:UPE_GPU_LIB_DIAG=$V/m3a2.so python bench.py --mode inplace $O" \
 "B0b:120:python bench.py $O" \
 "Bm1a2b:120:UPE_GPU_LIB_DIAG=$V/m1a2.so python bench.py $O" \
 "Bm1a1b:120:UPE_GPU_LIB_DIAG=$V/m1a1.so python bench.py $O" \
 "Bi0b:120:python bench.py --mode inplace $O" \
 "Bim3b:120:UPE_GPU_LIB_DIAG=$V/m3a2.so python bench.py --mode inplace $O" \
 "m1a1t:300:UPE_GPU_LIB_DIAG=$V/m1a1.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_neigh_paths.py $T"
