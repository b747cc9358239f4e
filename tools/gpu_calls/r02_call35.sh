# round 2: small-table lean kernels (rules always in LDS, rule_stats always in the replicated
# accumulators; config B) against the previous build, emit and in place; parity
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix"
T="-m gpu -x -q --timeout 200 --timeout-method thread"
bash tools/gpu_session.sh \
 "Bprev:120:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py $O" \
 "Bsmall:120:python bench.py $O" \
 "Bprevb:120:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py $O" \
 "Bsmallb:120:python bench.py $O" \
 "Biprev:120:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py $O --mode inplace" \
 "Bismall:120:python bench.py $O --mode inplace" \
 "Aprev:120:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py --config A $O" \
 "Asmall:120:python bench.py --config A $O" \
 "st:400:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py tests/test_gpu_dropin.py tests/test_gpu_batches.py tests/test_gpu_control.py tests/test_gpu_rss_egress.py $T"
