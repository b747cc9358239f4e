bash tools/gpu_session.sh \
 "trC4M:200:UPE_BENCH_TRACE=1 python bench.py --config C --packets 4194304 --no-cpu-baseline --no-hbm-probe --steps 100" \
 "trC4Mc20:200:UPE_BENCH_TRACE=1 python bench.py --config C --packets 4194304 --no-cpu-baseline --no-hbm-probe --steps 100 --max-copies 20" \
 "trB:200:UPE_BENCH_TRACE=1 python bench.py --no-cpu-baseline --no-hbm-probe"
