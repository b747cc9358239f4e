# round 2: HEAD check as the driver runs it (GPU tests, smoke, the driver's bench command)
bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json"
