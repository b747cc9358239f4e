# round 2: late-claim threshold (UPE_LATE_CLAIM: claim the next chunk only after finishing once
# fewer than this many of the workgroup's chunks are unclaimed) re-swept with the mid-chunk
# prefetch, B and C
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix"
bash tools/gpu_session.sh \
 "B16:120:python bench.py $O" \
 "B0:120:UPE_GPU_LIB_DIAG=$V/lc0.so python bench.py $O" \
 "B4:120:UPE_GPU_LIB_DIAG=$V/lc4.so python bench.py $O" \
 "B8:120:UPE_GPU_LIB_DIAG=$V/lc8.so python bench.py $O" \
 "B32:120:UPE_GPU_LIB_DIAG=$V/lc32.so python bench.py $O" \
 "C16:120:python bench.py --config C $O" \
 "C0:120:UPE_GPU_LIB_DIAG=$V/lc0.so python bench.py --config C $O" \
 "C4:120:UPE_GPU_LIB_DIAG=$V/lc4.so python bench.py --config C $O" \
 "C8:120:UPE_GPU_LIB_DIAG=$V/lc8.so python bench.py --config C $O" \
 "C32:120:UPE_GPU_LIB_DIAG=$V/lc32.so python bench.py --config C $O" \
 "B16b:120:python bench.py $O" \
 "B8b:120:UPE_GPU_LIB_DIAG=$V/lc8.so python bench.py $O" \
 "B4b:120:UPE_GPU_LIB_DIAG=$V/lc4.so python bench.py $O"
