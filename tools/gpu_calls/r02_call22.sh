# round 2: the driver's short bench (20 steps) after moving the batch-pointer array out of the
# timed region; where the host time of the timed region goes (UPE_BENCH_TRACE)
O="--no-cpu-baseline --no-hbm-probe"
bash tools/gpu_session.sh \
 "s20a:120:python bench.py --gpus 1 --steps 20 --warmup 5 $O" \
 "s20b:120:python bench.py --gpus 1 --steps 20 --warmup 5 $O" \
 "s20t:120:UPE_BENCH_TRACE=1 python bench.py --gpus 1 --steps 20 --warmup 5 --no-imix --no-other-mode $O" \
 "s200t:120:UPE_BENCH_TRACE=1 python bench.py --no-imix --no-other-mode $O"
