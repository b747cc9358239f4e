# round 2: the next chunk's window issued mid-chunk (after the rule match; UPE_MID_PREFETCH),
# at 1024 threads (4 waves/SIMD) and at 768 threads (3 waves/SIMD, 168 VGPRs), against the
# product build; B and C; parity of each variant
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix"
T="-m gpu -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh \
 "B0:120:python bench.py $O" \
 "Bmp1:120:UPE_GPU_LIB_DIAG=$V/mp1.so python bench.py $O" \
 "Bb768:120:UPE_GPU_LIB_DIAG=$V/b768.so python bench.py $O" \
 "Bb768mp:120:UPE_GPU_LIB_DIAG=$V/b768mp.so python bench.py $O" \
 "C0:120:python bench.py --config C $O" \
 "Cmp1:120:UPE_GPU_LIB_DIAG=$V/mp1.so python bench.py --config C $O" \
 "Cb768:120:UPE_GPU_LIB_DIAG=$V/b768.so python bench.py --config C $O" \
 "Cb768mp:120:UPE_GPU_LIB_DIAG=$V/b768mp.so python bench.py --config C $O" \
 "B0b:120:python bench.py $O" \
 "Bmp1b:120:UPE_GPU_LIB_DIAG=$V/mp1.so python bench.py $O" \
 "Bb768mpb:120:UPE_GPU_LIB_DIAG=$V/b768mp.so python bench.py $O" \
 "mp1t:300:UPE_GPU_LIB_DIAG=$V/mp1.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_neigh_paths.py $T" \
 "b768mpt:300:UPE_GPU_LIB_DIAG=$V/b768mp.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_neigh_paths.py $T"
