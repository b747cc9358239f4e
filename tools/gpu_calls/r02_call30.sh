# round 2: lean emit kernel (no flow_hash / length side array / in-memory neighbour lookups
# compiled in: SGPR spills 96 -> 70) against the product build, B and C; parity of the golden
# and full-size emit cases
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix"
T="-m gpu -x -q --timeout 200 --timeout-method thread"
bash tools/gpu_session.sh \
 "B0:120:python bench.py $O" \
 "Blean:120:UPE_GPU_LIB_DIAG=$V/lean.so python bench.py $O" \
 "C0:120:python bench.py --config C $O" \
 "Clean:120:UPE_GPU_LIB_DIAG=$V/lean.so python bench.py --config C $O" \
 "B0b:120:python bench.py $O" \
 "Bleanb:120:UPE_GPU_LIB_DIAG=$V/lean.so python bench.py $O" \
 "C0b:120:python bench.py --config C $O" \
 "Cleanb:120:UPE_GPU_LIB_DIAG=$V/lean.so python bench.py --config C $O" \
 "leant:300:UPE_GPU_LIB_DIAG=$V/lean.so python -u -m pytest tests/test_gpu_parity.py $T -k 'golden_no_control or full_size_digest or ragged'"
