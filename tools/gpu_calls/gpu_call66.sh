bash tools/gpu_session.sh \
 "h64k:200:python bench.py --host-reps 10 --host-chunk 65536 --no-cpu-baseline --no-hbm-probe --steps 20" \
 "h256k:200:python bench.py --host-reps 10 --host-chunk 262144 --no-cpu-baseline --no-hbm-probe --steps 20" \
 "h1m:200:python bench.py --host-reps 10 --host-chunk 1048576 --no-cpu-baseline --no-hbm-probe --steps 20" \
 "h4m:200:python bench.py --packets 4194304 --host-reps 6 --host-chunk 524288 --no-cpu-baseline --no-hbm-probe --steps 20"
