V=$PWD/build/var
bash tools/gpu_session.sh \
 "D:200:python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Dht256:200:UPE_GPU_LIB_DIAG=$V/ht256.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Dht2048:200:UPE_GPU_LIB_DIAG=$V/ht2048.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "tssT:300:python -u -m pytest tests/test_gpu_parity.py -x -q -k 'config_d or digest or kinds or tuple' --timeout 200 --timeout-method thread"
