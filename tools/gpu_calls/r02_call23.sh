# round 2: the driver's short bench with timing samples opened mid-period (not on the first
# call of the timed region), three times, and the default run
bash tools/gpu_session.sh \
 "s20a:120:python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-hbm-probe" \
 "s20b:120:python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-hbm-probe" \
 "s20c:120:python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-hbm-probe" \
 "s200:120:python bench.py --no-cpu-baseline --no-hbm-probe" \
 "emitt:300:python -u -m pytest tests/test_gpu_errors.py tests/test_gpu_batches.py -m gpu -x -q --timeout 120 --timeout-method thread"
