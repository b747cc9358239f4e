bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "benchB:300:python bench.py --config B" \
 "benchC:300:python bench.py --config C --no-cpu-baseline"
