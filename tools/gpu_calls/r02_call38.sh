# round 2: kernels without look-back, chosen once a launch reports agreeing L1 entries: GPU
# tests, then B / C / D against the previous build
V=$PWD/build/var
O="--no-cpu-baseline --no-hbm-probe --no-imix"
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "Bprev:120:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py $O" \
 "Bnew:120:python bench.py $O" \
 "Cprev:120:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py --config C $O" \
 "Cnew:120:python bench.py --config C $O" \
 "Bprevb:120:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py $O" \
 "Bnewb:120:python bench.py $O" \
 "Dprev:200:UPE_GPU_LIB_DIAG=$V/prev.so python bench.py --config D --steps 30 --warmup 3 --max-copies 4 $O" \
 "Dnew:200:python bench.py --config D --steps 30 --warmup 3 --max-copies 4 $O"
