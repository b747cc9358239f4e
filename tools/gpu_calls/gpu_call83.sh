V=$PWD/build/var
O="--config D --steps 20 --warmup 2 --max-copies 4 --no-cpu-baseline --no-hbm-probe --host-reps 0"
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread" \
 "profD:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profD5 -o p --output-format csv -- python bench.py $O" \
 "kl1:200:UPE_GPU_LIB_DIAG=$V/kl1.so python bench.py $O" \
 "kl2:200:UPE_GPU_LIB_DIAG=$V/kl2.so python bench.py $O" \
 "kl4:200:python bench.py $O" \
 "kl8:200:UPE_GPU_LIB_DIAG=$V/kl8.so python bench.py $O"
