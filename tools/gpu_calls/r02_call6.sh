# round 2: rule_stats group-by (config D, 64k rules) with 16 / 32 packets per thread per round
# (UPE_HIST_PER) against the product build's 8; parity of the config-D cases for both
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-other-mode --steps 30 --warmup 3 --max-copies 4"
bash tools/gpu_session.sh \
 "def_D:200:python bench.py --config D $O" \
 "hp16_D:200:UPE_GPU_LIB_DIAG=$V/hp16.so python bench.py --config D $O" \
 "hp32_D:200:UPE_GPU_LIB_DIAG=$V/hp32.so python bench.py --config D $O" \
 "def_D2:200:python bench.py --config D $O" \
 "hp16_D2:200:UPE_GPU_LIB_DIAG=$V/hp16.so python bench.py --config D $O" \
 "hp32_D2:200:UPE_GPU_LIB_DIAG=$V/hp32.so python bench.py --config D $O" \
 "hp16t:300:UPE_GPU_LIB_DIAG=$V/hp16.so python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k 'config_d or digest or kinds' --timeout 200 --timeout-method thread" \
 "hp32t:300:UPE_GPU_LIB_DIAG=$V/hp32.so python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k 'config_d or digest or kinds' --timeout 200 --timeout-method thread" \
 "profD16:300:UPE_GPU_LIB_DIAG=$V/hp16.so rocprofv3 --kernel-trace --stats -d gpurun_out/profD16 -o p --output-format csv -- python bench.py --config D $O"
