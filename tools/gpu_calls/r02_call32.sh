# round 2: lean in-place kernel (B/C --mode inplace) against the previous build, and with the
# mid-chunk prefetch in place too (UPE_MID_PREFETCH=3); parity of the in-place cases
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix --mode inplace"
T="-m gpu -x -q --timeout 200 --timeout-method thread"
bash tools/gpu_session.sh \
 "Bprev:120:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py $O" \
 "Blean:120:python bench.py $O" \
 "Bm3:120:UPE_GPU_LIB_DIAG=$V/m3.so python bench.py $O" \
 "Cprev:120:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py --config C $O" \
 "Clean:120:python bench.py --config C $O" \
 "Cm3:120:UPE_GPU_LIB_DIAG=$V/m3.so python bench.py --config C $O" \
 "Bprevb:120:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py $O" \
 "Bleanb:120:python bench.py $O" \
 "Bm3b:120:UPE_GPU_LIB_DIAG=$V/m3.so python bench.py $O" \
 "leant:400:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_neigh_paths.py tests/test_gpu_host.py tests/test_gpu_dropin.py $T"
