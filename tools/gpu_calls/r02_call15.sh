# round 2: mid-chunk window prefetch in the tuple-space emit kernel too (UPE_MID_PREFETCH=5),
# config D, with the config-D parity cases
V=$PWD/build/var
O="--config D --no-cpu-baseline --no-hbm-probe --no-other-mode --steps 30 --warmup 3 --max-copies 4"
T="-m gpu -x -q --timeout 200 --timeout-method thread"
bash tools/gpu_session.sh \
 "D0:200:python bench.py $O" \
 "Dm5:200:UPE_GPU_LIB_DIAG=$V/m5.so python bench.py $O" \
 "D0b:200:python bench.py $O" \
 "Dm5b:200:UPE_GPU_LIB_DIAG=$V/m5.so python bench.py $O" \
 "m5t:300:UPE_GPU_LIB_DIAG=$V/m5.so python -u -m pytest tests/test_gpu_parity.py $T -k 'config_d or digest or kinds'"
