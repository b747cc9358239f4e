V=$PWD/build/var
O="--config C --no-cpu-baseline --no-hbm-probe --host-reps 0"
bash tools/gpu_session.sh \
 "baseC:120:python bench.py $O" \
 "arp2kC:120:UPE_GPU_LIB_DIAG=$V/arp2k.so python bench.py $O" \
 "baseC2:120:python bench.py $O" \
 "arp2kC2:120:UPE_GPU_LIB_DIAG=$V/arp2k.so python bench.py $O"
