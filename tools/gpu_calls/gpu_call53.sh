bash tools/gpu_session.sh \
 "A:200:python bench.py --config A" \
 "hostA:200:python bench.py --config A --host-reps 10 --no-cpu-baseline --no-hbm-probe"
