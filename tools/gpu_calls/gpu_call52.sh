V=$PWD/build/var
bash tools/gpu_session.sh \
 "D:200:python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Dhd:200:UPE_GPU_LIB_DIAG=$V/hdirect.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "hdt:300:UPE_GPU_LIB_DIAG=$V/hdirect.so python -u -m pytest tests/test_gpu_parity.py -x -q -k 'config_d or digest or kinds' --timeout 200 --timeout-method thread"
