# round 2: the upper half of each workgroup's waves issue their first window in the prologue
# while the lower half stage the LDS tables (UPE_EARLY_WIN=1); B / C, parity; and the new
# ragged-size parity test on the product build
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix"
T="-m gpu -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh \
 "B0:120:python bench.py $O" \
 "Bewh:120:UPE_GPU_LIB_DIAG=$V/ewh.so python bench.py $O" \
 "C0:120:python bench.py --config C $O" \
 "Cewh:120:UPE_GPU_LIB_DIAG=$V/ewh.so python bench.py --config C $O" \
 "B0b:120:python bench.py $O" \
 "Bewhb:120:UPE_GPU_LIB_DIAG=$V/ewh.so python bench.py $O" \
 "C0b:120:python bench.py --config C $O" \
 "Cewhb:120:UPE_GPU_LIB_DIAG=$V/ewh.so python bench.py --config C $O" \
 "ragged:300:python -u -m pytest tests/test_gpu_parity.py $T -k ragged" \
 "ewht:300:UPE_GPU_LIB_DIAG=$V/ewh.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_neigh_paths.py $T"
