# round 2: the no-look-back kernel's residency census done with the first launch's (not at the
# switch): the driver's 20-step bench three times, the default once, GPU tests
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "s20a:300:python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s20a.json" \
 "s20b:300:python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/s20b.json" \
 "s20c:300:python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/s20c.json" \
 "s200:300:python bench.py --no-cpu-baseline > gpurun_out/s200.json"
