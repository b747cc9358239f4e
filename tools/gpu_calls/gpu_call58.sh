V=$PWD/build/var
bash tools/gpu_session.sh \
 "Dht2048:200:UPE_GPU_LIB_DIAG=$V/ht2048.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Dht4096:200:UPE_GPU_LIB_DIAG=$V/ht4096.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3" \
 "Dht8192:200:UPE_GPU_LIB_DIAG=$V/ht8192.so python bench.py --config D --no-cpu-baseline --no-hbm-probe --steps 30 --warmup 3"
