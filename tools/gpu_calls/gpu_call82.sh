O="--no-cpu-baseline --no-hbm-probe --host-reps 0"
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "profD:300:rocprofv3 --kernel-trace --stats -d gpurun_out/profD4 -o p --output-format csv -- python bench.py --config D --steps 20 --warmup 2 --max-copies 4 $O" \
 "D2:200:python bench.py --config D --steps 20 --warmup 2 --max-copies 4 $O"
