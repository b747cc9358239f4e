# round 2: one register set for the window on both loop paths (no copies of the prefetched one)
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix"
bash tools/gpu_session.sh \
 "B0:120:python bench.py $O" \
 "Bnc:120:UPE_GPU_LIB_DIAG=$V/nc.so python bench.py $O" \
 "B0b:120:python bench.py $O" \
 "Bncb:120:UPE_GPU_LIB_DIAG=$V/nc.so python bench.py $O" \
 "C0:120:python bench.py --config C $O" \
 "Cnc:120:UPE_GPU_LIB_DIAG=$V/nc.so python bench.py --config C $O"
