bash tools/gpu_session.sh \
 "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "benchB:200:python bench.py --no-cpu-baseline --no-hbm-probe"
