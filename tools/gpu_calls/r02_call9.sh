# round 2: config D ablations on the current kernel (diagnostic builds, results wrong by design):
# 1 no rule match, 2 no neighbour lookup, 4 no rule_stats, 8 no output stores
V=$PWD/build/var
O="--config D --no-cpu-baseline --no-hbm-probe --no-other-mode --steps 30 --warmup 3 --max-copies 4"
bash tools/gpu_session.sh \
 "D0:200:python bench.py $O" \
 "Da1:200:UPE_GPU_LIB_DIAG=$V/a1.so python bench.py $O" \
 "Da2:200:UPE_GPU_LIB_DIAG=$V/a2.so python bench.py $O" \
 "Da4:200:UPE_GPU_LIB_DIAG=$V/a4.so python bench.py $O" \
 "Da8:200:UPE_GPU_LIB_DIAG=$V/a8.so python bench.py $O" \
 "B0:200:python bench.py --no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix" \
 "Ba1:200:UPE_GPU_LIB_DIAG=$V/a1.so python bench.py --no-cpu-baseline --no-hbm-probe --no-other-mode --no-imix" \
 "Ca1:200:UPE_GPU_LIB_DIAG=$V/a1.so python bench.py --config C --no-cpu-baseline --no-hbm-probe --no-other-mode"
