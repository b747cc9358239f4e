bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "benchD:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profD -o p --output-format csv -- python bench.py --config D --steps 20 --warmup 2 --no-cpu-baseline --max-copies 4 --host-reps 3" \
 "benchB:300:python bench.py --config B --no-cpu-baseline --host-reps 0"
